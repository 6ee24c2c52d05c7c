"""Out of device memory fails the call cleanly.

The reference's alloc_padded does not check its calloc (/root/reference/lib/hash/utility.cpp:50);
the C-ABI promises S3H_ENOMEM with a message naming the allocation, and no damage to later
calls.  HBM is filled with torch allocations until less than 512 MiB (then less than 48 MiB)
is free, and the entry points are driven into their allocation failures:

  * a plan too large for what is left              -> S3H_ENOMEM "plan alloc (... slots ...)"
  * a stream object of 10^8 messages               -> S3H_ENOMEM
  * the host path on C2-sized parts (768 MiB ring at full size) with < 512 MiB free: the ring
    is sized to a quarter of the free HBM (capi.hip run_host_shard), so the call SUCCEEDS with
    smaller slices and bit-exact digests -- by design, a busy GPU still hashes;
  * the host path on 4M parts of 64 B with < 48 MiB free: they go in groups (capi.hip
    run_host_groups, whose two group buffers also shrink to a quarter of the free HBM), but
    their 128 MiB of digests cannot fit           -> S3H_ENOMEM "ensure_digests" (or the
    group buffers / plans when those fail first)

After every failure a small device batch on the remaining memory must still be bit-exact (a
failed allocation must not leak into a later launch's error check), and once the memory is
given back the same calls succeed and match the oracle, the host path reusing its context.
"""
import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
MIB = 1 << 20
S3H_ENOMEM = -4
SEED = 20241008


def _fill(torch, dev, leave: int, hog: list) -> int:
    """Allocate device memory into `hog` until less than `leave` bytes are free; returns free."""
    chunk = 16 << 30
    while chunk >= 2 * MIB:
        free, _ = torch.cuda.mem_get_info(dev)
        if free - chunk < leave // 2:
            chunk //= 2
            continue
        try:
            hog.append(torch.empty(chunk, dtype=torch.uint8, device=dev))
        except torch.OutOfMemoryError:
            chunk //= 2
        if torch.cuda.mem_get_info(dev)[0] < leave:
            break
    return torch.cuda.mem_get_info(dev)[0]


def _small_batch_ok(torch, dev, oracle, rng):
    lens = rng.integers(0, 5000, 100)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.uint64)
    host = rng.integers(0, 256, int(lens.sum()) + 64, dtype=np.uint8)
    got = s3.sha256_batch_device(torch.from_numpy(host).to(dev), offs, lens)
    assert np.array_equal(got.cpu().numpy().view(np.uint32), oracle.batch(host, offs, lens))


def _enomem(fn, *names):
    with pytest.raises(s3.S3HashError) as e:
        fn()
    assert e.value.code == S3H_ENOMEM, str(e.value)
    assert any(n in str(e.value) for n in names), str(e.value)
    return str(e.value)


def test_out_of_hbm_fails_cleanly_and_recovers(torch_cuda, oracle):
    torch = torch_cuda
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(31)
    n, L = 1024, 8 * MIB
    lens = np.full(n, L, dtype=np.uint64)
    offs = np.arange(n, dtype=np.uint64) * np.uint64(L)
    data = torch.empty(n * L, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, np.arange(n), SEED)
    want = s3.sha256_batch_device(data, offs, lens).cpu().numpy().view(np.uint32)
    host = s3.PinnedBuffer(n * L, s3.device_numa(0)["node"])
    torch.from_numpy(host.array).copy_(data)
    del data
    parts = s3.BufferParts(host.array, offs, lens)
    tiny_n = 4 << 20
    tiny = rng.integers(0, 256, tiny_n * 64, dtype=np.uint8)
    tiny_offs = np.arange(tiny_n, dtype=np.uint64) * np.uint64(64)
    tiny_lens = np.full(tiny_n, 64, dtype=np.uint64)
    tiny_parts = s3.BufferParts(tiny, tiny_offs, tiny_lens)
    big = 50_000_000  # 1 GB of plan slots + order
    big_offs = np.zeros(big, dtype=np.uint64)
    msgs = {}
    s3.trim()  # no cached ring: the host path must allocate under pressure
    torch.cuda.empty_cache()
    hog: list = []
    try:
        free = _fill(torch, dev, 512 * MIB, hog)
        assert free < 512 * MIB, free
        msgs["plan"] = _enomem(lambda: s3.Plan(big_offs, big_offs), "plan alloc")
        assert "slots" in msgs["plan"]
        _small_batch_ok(torch, dev, oracle, rng)
        msgs["stream"] = _enomem(lambda: s3.Stream(100_000_000, device=0), "plan alloc", "stream")
        _small_batch_ok(torch, dev, oracle, rng)
        # C2 parts with < 512 MiB of HBM: the ring shrinks to a quarter of it, digests exact
        assert np.array_equal(s3.sha256_batch_host(parts, ndevices=1), want)
        s3.trim()
        free = _fill(torch, dev, 48 * MIB, hog)
        assert free < 48 * MIB, free
        msgs["host"] = _enomem(lambda: s3.sha256_batch_host(tiny_parts, ndevices=1),
                               "host ring", "host group", "plan alloc", "ensure_digests")
        _small_batch_ok(torch, dev, oracle, rng)
        msgs["host_again"] = _enomem(lambda: s3.sha256_batch_host(tiny_parts, ndevices=1),
                                     "host ring", "host group", "plan alloc", "ensure_digests")
    finally:
        del hog
        torch.cuda.empty_cache()
    # memory back: the same calls succeed, the host context is rebuilt and then reused
    for _ in range(2):
        assert np.array_equal(s3.sha256_batch_host(parts, ndevices=1), want)
    got = s3.sha256_batch_host(tiny_parts, ndevices=1)
    assert np.array_equal(got, oracle.batch(tiny, tiny_offs, tiny_lens))
    with s3.Stream(1_000_000, device=0) as st:  # a large stream object fits again
        d = st.final()  # 10^6 empty messages
    assert (d == oracle.sha256(b"")).all()
    _small_batch_ok(torch, dev, oracle, rng)
    print({k: v[:160] for k, v in msgs.items()})
