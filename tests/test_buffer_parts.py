"""BufferParts: host parts as (offset, length) ranges of one buffer (CPU checks of the
pointer arithmetic and bounds; the GPU digests are compared in tests/test_gpu_host.py)."""
import numpy as np
import pytest
import torch

import s3client_amd as s3
from s3client_amd import hashing


def test_pointers_are_base_plus_offset_and_null_for_empty_parts():
    buf = np.arange(4096, dtype=np.uint8)
    bp = s3.BufferParts(buf, [0, 100, 4000, 7], [100, 0, 96, 0])
    keep, ptrs, lens = hashing._host_parts(bp)
    assert len(bp) == 4 and keep is bp
    base = buf.ctypes.data
    assert [ptrs[i] for i in range(4)] == [base, None, base + 4000, None]
    assert lens.tolist() == [100, 0, 96, 0]


def test_torch_host_tensor_and_bounds():
    t = torch.zeros(1000, dtype=torch.uint8)
    assert int(s3.BufferParts(t, [10], [990]).addrs[0]) == t.data_ptr() + 10
    for offs, lens in (([995], [10]), ([2**64 - 1], [2]), ([1001], [0 + 1])):
        with pytest.raises(ValueError):
            s3.BufferParts(t, offs, lens)
    s3.BufferParts(t, [5000], [0])  # an empty part may point anywhere
    with pytest.raises(ValueError):
        s3.BufferParts(t[::2], [0], [1])  # not contiguous
    with pytest.raises(ValueError):
        s3.BufferParts(np.zeros(10, np.uint8), [0, 1], [1])
