"""The gfx950 code object libs3hash.so ships (CPU only: read from the library file).

* Every flag-synchronised kernel (two-group skew, shared-SIMD skew, both dual-digest group
  kernels) contains the global atomic OR with which a timed-out producer/consumer wait reports
  into the device error word (sha256_kernels.hip flag_wait_ge) -- so the host entry points
  that read the word can fail the call instead of returning wrong digests.  The forced-fault
  library (tests/cpp/build/libs3hash_stall.so) is exercised on the GPU by test_gpu_errors.py.
* s3client_amd/kernel_isa_counts.json (bench.py's instruction counts and the code hashes that
  key profiles/*_pmc.json) describes THIS library's code object.
* Host staging threads follow the CPUs the process may use (s3h_host_threads).
"""
import json
import math
import os
import sys

import pytest

from s3client_amd import _native
import s3client_amd as s3

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import code_object  # noqa: E402
import isa_counts  # noqa: E402


@pytest.fixture(scope="module")
def shipped():
    return code_object.disassemble(_native.LIB_PATH)


def _atomics(lines, sym):
    return sum(bool(isa_counts.ERR_STORE.match(l)) for l in code_object.function_body(lines, sym))


@pytest.mark.parametrize("kernel", isa_counts.FLAG_KERNELS)
def test_flag_kernels_store_the_error_word(shipped, kernel):
    assert _atomics(shipped, isa_counts.ALL_KERNELS[kernel]) >= 1, kernel


def test_barrier_kernels_have_no_error_store(shipped):
    # kernels synchronised by s_barrier cannot time out: nothing to report
    for k in ("skew", "skewp", "pc", "lane", "md5-pc"):
        assert _atomics(shipped, isa_counts.ALL_KERNELS[k]) == 0, k


def test_isa_counts_describe_the_shipped_library(shipped):
    with open(os.path.join(ROOT, "s3client_amd", "kernel_isa_counts.json")) as f:
        counts = json.load(f)
    for k, sym in isa_counts.ALL_KERNELS.items():
        assert counts["code_hash"][k] == code_object.code_hash(shipped, sym), k
    for k in isa_counts.FLAG_KERNELS:
        assert counts["error_word_atomics"][k] >= 1
    # the skew consumer's fast loop: the round stream plus LDS reads, nothing of the cold
    # error-report span (tools/isa_counts.py loops())
    assert 540 < counts["kernels"]["skew"]["instr_per_block"] < 550
    assert 540 < counts["kernels"]["skews"]["instr_per_block"] < 550


def test_code_hash_ignores_label_numbering():
    a = ["\ts_branch L7   // 0: 00", "0000000000000010 <L7>:", "\tv_add_u32_e32 v1, v2, v3   // 10: 00"]
    b = ["\ts_branch L9   // 8: 11", "0000000000000018 <L9>:", "\tv_add_u32_e32 v1, v2, v3   // 18: 11"]
    assert code_object.instructions(a) == code_object.instructions(b)


def _expected_cpus():
    n = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        quota = None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / per if q > 0 else None
        except (OSError, ValueError):
            pass
    return min(n, max(1, math.ceil(quota))) if quota else n


def test_host_threads_follow_affinity_and_quota():
    cpus = _expected_cpus()
    for nd in (1, 2, 3, 8, 64):
        per, got = s3.host_threads(nd)
        assert got == cpus
        assert per == min(16, max(1, cpus // nd))
        assert per * nd <= max(cpus, nd)  # never more threads than CPUs (1 per device minimum)


def test_host_threads_respect_a_narrowed_affinity():
    # a child process pinned to 2 CPUs must see 2 (or fewer under a smaller quota)
    import subprocess
    code = ("import os,sys;os.sched_setaffinity(0,sorted(os.sched_getaffinity(0))[:2]);"
            "sys.path.insert(0,'.');import s3client_amd as s;print(*s.host_threads(1))")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, cwd=ROOT)
    assert r.returncode == 0, r.stderr
    per, cpus = map(int, r.stdout.split())
    assert cpus == min(2, _expected_cpus()) and per == cpus


def test_pmc_profiles_carry_provenance_and_bench_checks_it():
    """Every newest profiles/r*_<cfg>_<kernel>_pmc.json records the kernel it measured (isa key
    + code hash), the library sha256 and the commit; bench.py takes its traffic only for a
    build running the same kernel machine code and returns null with the reason otherwise."""
    import glob
    import bench
    newest = {}
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_*_pmc.json"))):
        parts = os.path.basename(f).split("_")
        newest[(parts[1], "_".join(parts[2:-1]))] = f
    with open(os.path.join(ROOT, "s3client_amd", "kernel_isa_counts.json")) as fh:
        shipped = json.load(fh)["code_hash"]
    for (cfg, kname), f in newest.items():
        if os.path.basename(f)[:3] in ("r01", "r02"):
            continue  # round 1-2 summaries predate provenance (bench gives them null traffic)
        with open(f) as fh:
            s = json.load(fh)
        for k in ("kernel_key", "kernel_code_hash", "library_sha256", "git_head"):
            assert s.get(k), (f, k)
        key = s["kernel_key"]
        t, src, note = bench.pmc_traffic(cfg, kname, key, s["kernel_code_hash"], 1e9)
        assert t is not None and src.endswith(os.path.basename(f)), note
        t2, _, note2 = bench.pmc_traffic(cfg, kname, key, "0" * 16, 1e9)
        assert t2 is None and "0000000000000000" in note2
        if shipped.get(key) == s["kernel_code_hash"]:
            assert 0.999 < t / 1e9 < 1.01, (f, t)  # no re-reads: traffic == algorithmic bytes


def test_no_kernel_uses_scratch():
    """Every kernel of the shipped code object runs without scratch memory and without VGPR
    spills: a spill or a dynamically indexed register array (the MD5 producer's M+K rows once
    fell back to one when its loop outgrew the unroller) would put a memory round trip on
    the chains."""
    md = code_object.kernel_metadata(_native.LIB_PATH)
    assert len(md) >= 15
    for sym, m in md.items():
        assert m["private_segment_fixed_size"] == 0, (sym, m)
        assert m["vgpr_spill_count"] == 0, (sym, m)


@pytest.mark.parametrize("flags,ok", [([], True), (["-DS3H_EXP_SOLO=3"], False),
                                      (["-DS3H_EXP_MD5_BPS=2"], False),
                                      (["-DS3H_EXP_NONTEMPORAL_FETCH"], False),
                                      (["-DS3H_EXPERIMENT_BUILD", "-DS3H_EXP_SOLO=3",
                                        "-DS3H_EXP_MD5_BPS=2"], True)])
def test_product_build_refuses_experiment_switches(tmp_path, flags, ok):
    """exp_config.hpp: a build without S3H_EXPERIMENT_BUILD (the shipped libs3hash.so) must keep
    every experiment switch at its product value -- the kernels measured in DESIGN.md and
    hashed in kernel_isa_counts.json; `make exp` / `make stall` builds opt out explicitly."""
    import subprocess
    src = tmp_path / "t.cpp"
    src.write_text('#include "exp_config.hpp"\nint main() { return S3H_EXP_MD5_BPS; }\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only",
                        "-I" + os.path.join(ROOT, "s3client_amd", "csrc"), *flags, str(src)],
                       capture_output=True, text=True)
    assert (r.returncode == 0) == ok, r.stderr[-1500:]


def test_power_sampler_reports_instead_of_failing():
    """tools/power.py (bench's board-power sample): on a host without that GPU it reports an
    error in its summary instead of raising, and summarises samples as documented."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from power import PowerSampler
    with PowerSampler("0000:ff:1f.7", period=0.01) as ps:
        pass
    assert "error" in ps.summary()
    ps = PowerSampler("x")
    ps.samples = [(0.0, 300.0, 150.0), (0.1, 1300.0, 2300.0), (0.2, 1340.0, 2320.0)]
    s = ps.summary()
    assert s["samples"] == 3 and s["max_W"] == 1340.0 and s["busy_mean_W"] == 1320.0
    assert s["busy_clock_MHz_mean"] == 2310.0
