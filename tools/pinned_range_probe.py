#!/usr/bin/env python3
"""Which HIP runtime query tells whether [p, p+n) lies inside ONE page-locked allocation
(advisor r5: the group pipeline may DMA a whole increasing range of pinned parts at once only
then).  For a torch pinned buffer (hipHostMalloc), an s3h_host_alloc buffer (mmap +
hipHostRegister) and two separately pinned buffers, prints what hipMemGetAddressRange,
hipPointerGetAttribute(RANGE_START_ADDR / RANGE_SIZE) and hipPointerGetAttributes return for
interior pointers.  One JSON object per line."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
import s3client_amd as s3  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemGetAddressRange.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t), ctypes.c_void_p]
hip.hipPointerGetAttribute.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, HIP_POINTER_ATTRIBUTE_RANGE_SIZE = 11, 12  # hip_runtime_api.h


def probe(name, base, size):
    for off in (0, 4096 + 13, size - 1):
        p = base + off
        b, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc1 = hip.hipMemGetAddressRange(ctypes.byref(b), ctypes.byref(n), ctypes.c_void_p(p))
        rs, rz = ctypes.c_void_p(), ctypes.c_size_t()
        rc2 = hip.hipPointerGetAttribute(ctypes.byref(rs), HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, ctypes.c_void_p(p))
        rc3 = hip.hipPointerGetAttribute(ctypes.byref(rz), HIP_POINTER_ATTRIBUTE_RANGE_SIZE, ctypes.c_void_p(p))
        print(json.dumps({"buffer": name, "base": hex(base), "size": size, "offset": off,
                          "memGetAddressRange": [rc1, hex(b.value or 0), n.value],
                          "range_start": [rc2, hex(rs.value or 0)], "range_size": [rc3, rz.value]}))
    hip.hipGetLastError()


t = torch.empty(3 << 20, dtype=torch.uint8, pin_memory=True)
probe("torch_pinned", t.data_ptr(), t.numel())
pb = s3.PinnedBuffer(3 << 20)
probe("s3h_host_alloc_runtime", pb.ptr, pb.nbytes)
pn = s3.PinnedBuffer(3 << 20, s3.device_numa(0)["node"])
probe("s3h_host_alloc_node", pn.ptr, pn.nbytes)
