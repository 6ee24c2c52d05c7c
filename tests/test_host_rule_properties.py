"""Property tests (hypothesis) of the host-side rules that need no GPU: the SHA-256 + MD5
mixed-grid layout (s3h_dual_layout = capi.hip dual_mixed_solo) and AUTO's route estimate
(s3h_route_estimate_ex = route.hpp route_choose).  The unit tests pin chosen shapes; these
check the rules' invariants over random batches."""
import heapq

import numpy as np
from hypothesis import given, settings, strategies as st

import s3client_amd as s3

MIB = 1 << 20
SKEW, SKEWP = 8, 32  # parts per skew group / per skewp group (capi.hip kSkew / kSkewp)


def batch(seed, n, shape):
    """A ragged batch of n parts: C3-like uniform 5-64 MiB, bimodal, or a few giants."""
    rng = np.random.default_rng(seed)
    if shape == "uniform":
        return (5 * MIB + rng.integers(0, 59 * MIB + 1, n)).tolist()
    if shape == "bimodal":
        return np.where(rng.random(n) < 0.1, 64 * MIB, rng.integers(MIB, 8 * MIB, n)).tolist()
    out = rng.integers(0, 4 * MIB, n)
    out[rng.integers(0, n, 1 + n // 500)] = 64 * MIB
    return out.tolist()


@settings(max_examples=60, deadline=None)
@given(st.integers(0, 2**32), st.integers(1, 9000), st.sampled_from(["uniform", "bimodal", "giants"]),
       st.integers(64, 304))
def test_dual_layout_fits_the_cus(seed, n, shape, cus):
    """Whatever the batch, a mixed grid (F > 0) exists only for 2,049 - 32 x CUs parts, leaves
    some parts to the skewp groups, and fits one workgroup per CU in the form it reports."""
    lengths = batch(seed, n, shape)
    F, apart = s3.dual_layout(lengths, cus=cus)
    if F == 0:
        assert not apart
        return
    assert 2048 < n <= SKEWP * cus
    assert F * SKEW < n
    wgs = F + -(-(n - F * SKEW) // SKEWP) + (-(-(SKEW * F) // 64) if apart else 0)
    assert wgs <= cus


def test_dual_layout_takes_both_forms_over_c3_shapes():
    """Over C3-like batches both forms occur: the apart form while it fits, round 3's beyond."""
    forms = {s3.dual_layout(batch(k, n, "uniform"))[1] for k, n in enumerate(range(2100, 8192, 350))}
    assert forms == {True, False}


@settings(max_examples=30, deadline=None)
@given(st.integers(1, 8), st.integers(2049, 8192))
def test_dual_layout_equal_lengths_keep_the_group_kernel(scale, n):
    assert s3.dual_layout([scale * MIB] * n) == (0, False)


MODEL = dict(cpu_bytes_per_s=2.5e9, chain_bytes_per_s=69e6, h2d_bytes_per_s=55e9, call_s=1.5e-4,
             cpu_threads=16, devices=1, cpu_all_bytes_per_s=37.5e9, staged_bytes_per_s=45e9)


def lpt(lengths, k):
    """Longest-first list schedule on k threads (the makespan route.hpp models)."""
    loads = [0] * k
    for x in sorted(lengths, reverse=True):
        heapq.heapreplace(loads, loads[0] + x)
    return max(loads)


@settings(max_examples=80, deadline=None)
@given(st.lists(st.integers(0, 64 * MIB), min_size=1, max_size=300),
       st.integers(1, 64), st.sampled_from(["pinned", "pageable", "file"]))
def test_route_estimate_matches_its_formula(lengths, threads, source):
    """The estimates are exactly the documented formulas (include/s3hash.h), and the route is
    the smaller one."""
    m = {**MODEL, "cpu_threads": threads}
    route, g, c = s3.route_estimate(lengths, m, source=source)
    total, longest, n = sum(lengths), max(lengths), len(lengths)
    feed = m["h2d_bytes_per_s"] if source == "pinned" else min(m["h2d_bytes_per_s"], m["staged_bytes_per_s"])
    want_g = m["call_s"] + max(longest / m["chain_bytes_per_s"], total / feed)
    k = min(n, threads)
    per_thread = min(k * m["cpu_bytes_per_s"], m["cpu_all_bytes_per_s"]) / k
    want_c = lpt(lengths, k) / per_thread
    assert np.isclose(g, want_g, rtol=1e-12, atol=1e-15)
    assert np.isclose(c, want_c, rtol=1e-12, atol=1e-15)
    assert route == ("cpu" if c < g else "gpu")
    # no schedule beats the larger of the longest part and an even split
    assert c >= max(longest, total / k) / per_thread * (1 - 1e-12)


@settings(max_examples=40, deadline=None)
@given(st.integers(1, 2000), st.integers(1, 16 * MIB))
def test_route_estimate_is_monotone_in_the_batch(n, part):
    """More parts of the same size never make either estimate shorter."""
    _, g1, c1 = s3.route_estimate([part] * n, MODEL)
    _, g2, c2 = s3.route_estimate([part] * (n + 1), MODEL)
    assert g2 >= g1 and c2 >= c1


def split_ref_tg(lengths, m, tg, ndevices=0, source="pinned"):
    """The split route's plan for one split of the host threads, restated (include/s3hash.h
    s3h_route_split_estimate): parts by length descending (ties by index), the first k on the
    CPU, the rest on the GPU; None when tg leaves the CPU side no thread."""
    n = len(lengths)
    order = sorted(range(n), key=lambda i: -lengths[i])
    total = sum(lengths)
    T = m["cpu_threads"]
    cap = max(1, min(ndevices, m["devices"]) if ndevices > 0 else m["devices"])
    staged = source != "pinned"
    if staged and tg * cap >= T:
        return None
    tc = T - tg * cap if staged else T
    feed = min(m["h2d_bytes_per_s"], m["staged_bytes_per_s"] * tg / T) if staged else m["h2d_bytes_per_s"]
    kmax = min(n, tc)
    rows = []
    for k in range(1, n):
        cpu = [lengths[order[i]] for i in range(k)]
        t = min(k, kmax)
        if staged:
            per_thread = min(T * m["cpu_bytes_per_s"], m["cpu_all_bytes_per_s"]) / T
        else:
            per_thread = min(t * m["cpu_bytes_per_s"], m["cpu_all_bytes_per_s"]) / t
        c = lpt(cpu, kmax) / per_thread
        devs = max(1, min(n - k, cap))
        f = (total - sum(cpu)) / devs / feed
        g = m["call_s"] + max(lengths[order[k]] / m["chain_bytes_per_s"], f)
        rows.append((k, max(g, c), max(f, c)))
    smin = min(r[1] for r in rows)
    k, s_, _ = min((r for r in rows if r[1] <= smin * 1.005), key=lambda r: r[2])
    return s_, k


def split_ref(lengths, m, ndevices=0, source="pinned"):
    """The whole plan: tg = 0 for pinned parts, else the best of each device's share T / N of
    the host threads x {1, 4, 6, 8, 9} / 12 that leave the CPU side a thread (topology.cpp
    split_stage_candidates); many small pinned parts (the group pipeline packs them) are
    planned as staged."""
    if source == "pinned" and len(lengths) > 64 and (
            max(lengths) <= MIB or (len(lengths) > 256 and max(lengths) != min(lengths))):
        source = "pageable"
    if source == "pinned":
        s_, k = split_ref_tg(lengths, m, 0, ndevices, source)
        return s_, k, 0
    T = m["cpu_threads"]
    cap = max(1, min(ndevices, m["devices"]) if ndevices > 0 else m["devices"])
    best = None
    cands = dict.fromkeys(max(1, max(1, T // cap) * num // 12) for num in (1, 4, 6, 8, 9))
    for t in (t for t in cands if t * cap < T):
        r = split_ref_tg(lengths, m, t, ndevices, source)
        if r and (best is None or r[0] < best[0]):
            best = (r[0], r[1], t)
    return best


@settings(max_examples=80, deadline=None)
@given(st.lists(st.integers(0, 64 * MIB), min_size=1, max_size=60), st.integers(1, 24),
       st.integers(1, 8), st.sampled_from(["pinned", "pageable", "file"]))
def test_route_split_estimate_matches_its_formula(lengths, threads, devices, source):
    """The split plan is exactly the documented rule (the balanced m among those within 0.5 %
    of the minimum estimate), and a single part is not split."""
    m = {**MODEL, "cpu_threads": threads, "devices": devices}
    k, tg, s_ = s3.route_split_estimate(lengths, m, source=source)
    want = split_ref(lengths, m, source=source) if len(lengths) > 1 else None
    if want is None:  # one part, or no thread left for the CPU side
        assert (k, tg, s_) == (0, 0, 0.0)
        return
    want_s, want_k, want_tg = want
    assert 1 <= k < len(lengths)
    assert np.isclose(s_, want_s, rtol=1e-12, atol=1e-15)
    assert (k, tg) == (want_k, want_tg)


def test_route_split_on_c2_shapes():
    """C2 from pinned memory under the box's measured rates (profiles/r05_route_sweep.json): the
    split beats both single routes, bounded below by one 8 MiB chain; a batch of 8 parts (one
    job of upload.cpp) gains nothing from the GPU side."""
    m = dict(MODEL, cpu_bytes_per_s=2.4e9, cpu_all_bytes_per_s=39e9, chain_bytes_per_s=69e6,
             h2d_bytes_per_s=56e9, cpu_threads=16)
    lens = [8 * MIB] * 1024
    route, g, c = s3.route_estimate(lens, m)
    k, tg, s_ = s3.route_split_estimate(lens, m)
    assert route == "gpu" and s_ < 0.85 * min(g, c) and tg == 0
    assert s_ >= 8 * MIB / m["chain_bytes_per_s"]
    assert 350 < k < 500  # the feed balanced against the CPU side: 8 GiB x 39 / (39 + 56)
    route, g, c = s3.route_estimate(lens[:8], m)
    k, tg, s_ = s3.route_split_estimate(lens[:8], m)
    assert route == "cpu" and s_ >= c


def test_route_split_plans_small_pinned_parts_as_staged():
    """Many small pinned parts go through the group pipeline, whose copy threads pack them once
    the CPU side has taken parts out of their range, and more than 256 ragged pinned parts are
    staged: the split plan gives both staging threads, exactly as for pageable parts.  Equal
    large parts (DMA'd as they are) keep every thread for the CPU side."""
    lens = list(np.random.default_rng(3).integers(1, MIB, 500))
    m = {**MODEL, "cpu_threads": 16}
    assert s3.route_split_estimate(lens, m, source="pinned") == s3.route_split_estimate(lens, m, source="pageable")
    assert s3.route_split_estimate(lens, m, source="pinned")[1] > 0
    assert s3.route_split_estimate(lens[:-1] + [2 * MIB], m, source="pinned")[1] > 0
    assert s3.route_split_estimate([2 * MIB] * 500, m, source="pinned")[1] == 0
    assert s3.route_split_estimate(lens[:200] + [2 * MIB], m, source="pinned")[1] == 0
