"""Routing of both digests and the self-correcting route model on the GPU (VERDICT r5 items 1
and 3).

* Content-MD5 + x-amz-content-sha256 on every route -- GPU (one grid, one PCIe pass), CPU (both
  digests per part in one pass over memory), split and AUTO -- for C2-shape parts (1,024 x 8
  MiB) from pinned memory, pageable memory and a file, and a C3-like ragged set: every digest vs
  the oracle.  AUTO prices what it computes: its pick for both digests is s3h_route_choose's
  under the dual rates, not the SHA-256 one.
* The model is measured per device and per digest set; a model mispriced by a test hook
  (s3h_route_scale, "a model taken while the GPU was busy") returns to the faster route within
  a bounded number of calls: at once when the mispriced route is the one taken (its observed
  time diverges and the observed factor corrects it), after the refresh period when it is the
  route NOT taken (nothing to observe; the periodic re-measurement re-prices it).
"""
import numpy as np
import pytest

import s3client_amd as s3

pytestmark = pytest.mark.gpu
MIB = 1 << 20
SEED = 20241008


def _gen(torch, n, L, ragged=None):
    """n parts of L bytes (or lengths `ragged`) from generator G, packed 256-B aligned: (host
    numpy bytes, offsets, lengths)."""
    lens = np.full(n, L, dtype=np.uint64) if ragged is None else np.asarray(ragged, dtype=np.uint64)
    offs = np.concatenate([[0], np.cumsum((lens + 255) // 256 * 256)[:-1]]).astype(np.uint64)
    total = int(offs[-1] + lens[-1]) + 256
    dev = torch.empty(total, dtype=torch.uint8, device="cuda")
    s3.generate_parts(dev, offs, lens, np.arange(lens.size), SEED)
    host = dev.cpu().numpy()
    del dev
    torch.cuda.empty_cache()
    return host, offs, lens


@pytest.fixture(scope="module")
def c2(torch_cuda, oracle):
    host, offs, lens = _gen(torch_cuda, 1024, 8 * MIB)
    want_s = oracle.batch(host, offs, lens, threads=16)
    want_m = oracle.md5_batch(host, offs, lens, threads=16)
    return host, offs, lens, want_s, want_m


@pytest.mark.parametrize("source", ["pinned", "pageable", "file"])
def test_both_digests_every_route_c2(torch_cuda, c2, tmp_path, source):
    torch = torch_cuda
    host, offs, lens, want_s, want_m = c2
    if source == "file":
        path = tmp_path / "c2.bin"
        host.tofile(path)
    else:
        buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=source == "pinned")
        buf.numpy()[:] = host
        parts = s3.BufferParts(buf, offs, lens)
    rates = s3.route_rates()
    for route in ("gpu", "cpu", "split", "auto"):
        if source == "file":
            sha, m5, taken = s3.sha256_md5_file_parts_routed(str(path), offs, lens, route=route)
        else:
            sha, m5, taken = s3.sha256_md5_batch_routed(parts, route=route)
        assert taken == route or route == "auto", (route, taken)
        bad_s = np.flatnonzero((sha != want_s).any(axis=1))
        bad_m = np.flatnonzero((m5 != want_m).any(axis=1))
        assert bad_s.size == 0 and bad_m.size == 0, (source, route, bad_s[:8], bad_m[:8])
    # SHA-256 alone still routes and splits as before
    if source != "file":
        got, taken = s3.sha256_batch_routed(parts, route="split")
        assert taken == "split" and np.array_equal(got, want_s)
        m5, taken = s3.md5_batch_routed(parts, route="split")
        assert taken == "split" and np.array_equal(m5, want_m)
    assert rates["chain_bytes_per_s"][2] > 0 and rates["cpu_bytes_per_s"][1] > 0


def test_both_digests_ragged_c3_like(torch_cuda, oracle, tmp_path):
    """A ragged set (300 parts of U[1, 16] MiB, plus empty and tiny parts): both digests on
    every route from pinned and pageable memory and a file, vs the oracle."""
    torch = torch_cuda
    rng = np.random.default_rng(606)
    lens = rng.integers(1 * MIB, 16 * MIB, 300)
    lens[:4] = [0, 1, 55, 64]
    host, offs, lens = _gen(torch, 0, 0, ragged=lens)
    want_s = oracle.batch(host, offs, lens, threads=16)
    want_m = oracle.md5_batch(host, offs, lens, threads=16)
    path = tmp_path / "c3like.bin"
    host.tofile(path)
    for source in ("pinned", "pageable", "file"):
        if source != "file":
            buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=source == "pinned")
            buf.numpy()[:] = host
            parts = s3.BufferParts(buf, offs, lens)
        for route in ("gpu", "cpu", "split", "auto"):
            if source == "file":
                sha, m5, taken = s3.sha256_md5_file_parts_routed(str(path), offs, lens, route=route)
            else:
                sha, m5, taken = s3.sha256_md5_batch_routed(parts, route=route)
            assert np.array_equal(sha, want_s) and np.array_equal(m5, want_m), (source, route, taken)


def test_auto_prices_both_digests(torch_cuda, oracle):
    """AUTO's pick for both digests is s3h_route_choose's under the live rates for the dual
    digest set -- and, priced on the measured rates alone (corrections left by earlier calls
    reset to 1), for a batch the CPU wins on SHA-256 alone the dual pick is no longer the CPU
    (CPU MD5 + SHA-256 is ~3.5x slower per thread than SHA-NI SHA-256 alone)."""
    torch = torch_cuda
    host, offs, lens = _gen(torch, 256, 8 * MIB)
    buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=True)
    buf.numpy()[:] = host
    parts = s3.BufferParts(buf, offs, lens)
    want_s = oracle.batch(host, offs, lens, threads=16)
    want_m = oracle.md5_batch(host, offs, lens, threads=16)
    R = s3.route_rates()
    c_both = s3.route_choose(lens, R, "both")
    R0 = dict(R, gpu_factor=[1.0] * 3, cpu_factor=[1.0] * 3)
    c_sha0 = s3.route_choose(lens, R0, "sha256")
    c_both0 = s3.route_choose(lens, R0, "both")
    print("rates", R, "\nlive choice both", c_both, "\nmeasured-rate choices sha256", c_sha0,
          "both", c_both0)
    assert c_both0["cpu_s"] > 2.0 * c_sha0["cpu_s"]  # MD5 + SHA-256 per CPU thread
    sha, m5, taken = s3.sha256_md5_batch_routed(parts, route="auto")
    assert taken == c_both["route"]
    assert np.array_equal(sha, want_s) and np.array_equal(m5, want_m)
    got, taken_sha = s3.sha256_batch_routed(parts, route="auto")
    assert np.array_equal(got, want_s)
    if c_sha0["route"] == "cpu":
        assert c_both0["route"] != "cpu"


def test_device_rates_and_state():
    """Each device's chain and H2D rates are measured on their own; the model uses the slowest
    device; the state counts its measurements."""
    n = s3.device_count()
    R = s3.route_rates()
    assert R["version"] == 2 and R["size"] > 0 and R["devices"] == n
    chains, h2ds = [], []
    for d in range(n):
        ch, h = s3.route_device_rates(d, "sha256")
        assert 20e6 < ch < 1e9 and 5e9 < h < 200e9, (d, ch, h)
        chains.append(ch)
        h2ds.append(h)
        m, _ = s3.route_device_rates(d, "md5")
        b, _ = s3.route_device_rates(d, "both")
        assert m > ch * 1.2 and 0.5 * ch < b <= 1.2 * ch, (m, b, ch)  # MD5 chains run ~1.8x faster
    R = s3.route_rates()
    assert R["chain_bytes_per_s"][0] == pytest.approx(min(chains), rel=1e-12)
    assert R["h2d_bytes_per_s"] == pytest.approx(min(h2ds), rel=1e-12)
    assert R["measurements"] >= 1
    m = s3.route_model()  # the frozen round-5 struct reads the same SHA-256 rates
    assert m["chain_bytes_per_s"] == pytest.approx(R["chain_bytes_per_s"][0], rel=1e-12)


def _pick_flipping_batch(rates, which, factor, want_base, want_after):
    """A batch shape whose AUTO route is in want_base under `rates` and in want_after once
    rate `which` is scaled by `factor` (pure s3h_route_choose arithmetic)."""
    key = {"chain": "chain_bytes_per_s", "h2d": "h2d_bytes_per_s", "cpu": "cpu_bytes_per_s"}[which]
    scaled = dict(rates)
    v = rates[key]
    scaled[key] = [x * factor for x in v] if isinstance(v, list) else v * factor
    if which == "cpu":
        scaled["cpu_all_bytes_per_s"] = [x * factor for x in rates["cpu_all_bytes_per_s"]]
    for L in (8 * MIB, 4 * MIB, 2 * MIB):
        for n in (64, 96, 128, 192, 256, 320, 384, 512, 640, 768, 1024, 1536):
            if n * L > 8 << 30:
                continue
            b = s3.route_choose([L] * n, rates, "sha256")["route"]
            a = s3.route_choose([L] * n, scaled, "sha256")["route"]
            if b in want_base and a in want_after:
                return n, L, b, a
    return None


def _run_until(parts, want, base, limit):
    routes = []
    for _ in range(limit):
        got, taken = s3.sha256_batch_routed(parts, route="auto")
        assert np.array_equal(got, want)
        routes.append(taken)
        if len(routes) > 1 and taken == base:
            break
    return routes


def test_route_recovers_when_the_taken_route_is_mispriced(torch_cuda, oracle):
    """The GPU chain rate scaled 3x up (a model that thinks the GPU 3x faster): AUTO takes
    the GPU (or a split) for a batch the CPU hashes faster, observes the GPU side take ~3x its
    prediction, and returns to the CPU on the next calls."""
    torch = torch_cuda
    s3.route_refresh_calls(64)
    R = s3.route_rates()
    pick = _pick_flipping_batch(R, "chain", 3.0, ("cpu",), ("gpu", "split"))
    if pick is None:
        pytest.skip(f"no batch shape flips under a 3x chain rate with these rates: {R}")
    n, L, base, after = pick
    host, offs, lens = _gen(torch, n, L)
    buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=True)
    buf.numpy()[:] = host
    parts = s3.BufferParts(buf, offs, lens)
    want = oracle.batch(host, offs, lens, threads=16)
    s3.route_rates()  # any due re-measurement happens here, not on the first call below
    s3.route_scale("chain", 3.0)
    routes = _run_until(parts, want, base, 6)
    st = s3.route_rates()
    print(f"{n} x {L >> 20} MiB: {base} -> scaled chain x3 -> routes {routes}; state {st}")
    assert routes[0] == after, routes  # the hook took effect
    assert routes[-1] == base and len(routes) <= 3, routes
    assert st["divergences"] >= 1


def test_route_recovers_when_the_route_not_taken_is_mispriced(torch_cuda, oracle):
    """The GPU's rate scaled 3x down (as if measured while a kernel occupied it): AUTO keeps
    the CPU, whose time matches its prediction -- nothing diverges -- until the periodic
    re-measurement (every 4 calls here) re-prices the GPU, and AUTO returns to the GPU side."""
    torch = torch_cuda
    prev = s3.route_refresh_calls(4)
    try:
        R = s3.route_rates()
        pick = None
        for which in ("chain", "h2d"):
            pick = _pick_flipping_batch(R, which, 1 / 3, ("gpu", "split"), ("cpu",))
            if pick:
                break
        if pick is None:
            pytest.skip(f"no batch shape flips under a 3x slower GPU with these rates: {R}")
        n, L, base, after = pick
        host, offs, lens = _gen(torch, n, L)
        buf = torch.empty(host.size, dtype=torch.uint8, pin_memory=True)
        buf.numpy()[:] = host
        parts = s3.BufferParts(buf, offs, lens)
        want = oracle.batch(host, offs, lens, threads=16)
        m0 = s3.route_rates()["measurements"]  # start the period right after a measurement
        s3.route_scale(which, 1 / 3)
        routes = _run_until(parts, want, base, 8)
        st = s3.route_rates()
        now = s3.route_choose([L] * n, st, "sha256")["route"]
        print(f"{n} x {L >> 20} MiB: {base} -> scaled {which} /3 -> routes {routes}; "
              f"re-priced model chooses {now}; state {st}")
        assert routes[0] == after, routes
        # the periodic re-measurement (every 4 calls) happened and dropped the 1/3 scale
        assert st["measurements"] > m0, st
        key = {"chain": "chain_bytes_per_s", "h2d": "h2d_bytes_per_s"}[which]
        v, v0 = st[key], R[key]
        assert (v[0] if isinstance(v, list) else v) > 0.6 * (v0[0] if isinstance(v0, list) else v0), st
        # ... and from then on AUTO follows the re-priced model: back to the GPU side, unless the
        # re-measured rates and the observed CPU factor (a shared box's CPUs ran faster than
        # first measured) now put the CPU ahead of it -- the model's own choice, not the scale
        assert routes[-1] == now, (routes, now)
        assert now != base or len(routes) <= 6, routes
    finally:
        s3.route_refresh_calls(prev)
