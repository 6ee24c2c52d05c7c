#!/usr/bin/env python3
"""Benchmark: device-resident SHA-256 GiB/s over batches of 8 MiB upload parts (MI355X).

BASELINE.json metric: "device-resident SHA-256 GiB/s over 8 MiB parts; bit-exact digests vs
lib/hash".  One step = one launch of the batched kernel over the whole per-GPU batch, inputs
already resident in HBM (generated in place by generator G).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4] [--kernel auto|pc|lane]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

N>1: one process per GPU, parts sharded round-robin (global part p -> rank p % N, slot
p // N), per-GPU work fixed (weak scaling), no collective on the data path -- only a barrier
and a max-reduction of the timing.  Rank 0 prints ONE JSON line, which lists every rank's
device (PCI address) and how many distinct devices ran.  `python bench.py --gpus N` without a
launcher starts the N ranks itself (launch_ranks: a child torch.distributed.run, started
before this process makes any GPU call).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SEED = 20241008
MIB = 1 << 20
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
CLOCK_GHZ = 2.4                 # MI355X peak engine clock (used when no clock probe ran)
ISSUE_FLOOR_CPI = 4.0           # one wave: <= 1 instruction per 4 cycles (MI355X_MICROARCH.md)
# Instructions one chain's wave issues per 64-B block.  A wave issues at most one instruction
# per ~4 cycles: this, not HBM, bounds each part's chain.  The AUTO kernels' counts come from
# the shipped code object (make -> tools/isa_counts.py -> s3client_amd/kernel_isa_counts.json:
# the consumer's unrolled fast loop in the llvm-objdump disassembly / blocks per step); the
# rest are round-1 hand counts of their multi-block loops.
HAND_INSTR_PER_BLOCK = {"quad": 592, "pair": 672, "pc": 923, "lane": 1425, "md5-pc": 280}


def chain_instr_per_block(kname: str, quad_waves: int):
    """(instructions per block, source) for the kernel a plan runs."""
    key = "skew_nc2" if kname == "skew" and quad_waves == 2 else kname
    try:
        with open(os.path.join(ROOT, "s3client_amd", "kernel_isa_counts.json")) as f:
            k = json.load(f)["kernels"][key]
        return k["instr_per_block"], f"code object ({k['symbol']} loop {k['loop_label']})"
    except (OSError, KeyError):
        return HAND_INSTR_PER_BLOCK[kname], "round-1 hand count"


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=["c2", "c3", "c4"])
    ap.add_argument("--parts-per-gpu", type=int, default=0, help="override batch size")
    ap.add_argument("--part-bytes", type=int, default=0, help="override part size (sweeps)")
    ap.add_argument("--kernel", default="auto", choices=["auto", "skew", "skewp", "skews", "quad", "pair", "pc", "lane"])
    ap.add_argument("--algo", default="sha256", choices=["sha256", "md5"],
                    help="md5: the SURVEY 8(f) Content-MD5/ETag kernel (not the metric)")
    ap.add_argument("--cpu-sample-parts", type=int, default=1024)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--slice-bytes", type=int, default=0, help="host mode: bytes per part per slice")
    ap.add_argument("--mode", default="device",
                    choices=["device", "host", "stream", "dual", "host-dual"],
                    help="host: H2D-inclusive rate from pinned host memory; stream: the parts "
                         "appended chunk by chunk through s3h_stream_*; dual / host-dual: "
                         "SHA-256 + MD5 of every part in one pass (none of these is the metric)")
    ap.add_argument("--chunk-bytes", type=int, default=MIB, help="stream mode: bytes per append")
    ap.add_argument("--stream-source", default="device", choices=["device", "pinned", "pageable"],
                    help="stream mode: chunks already in HBM (update_device) or in host memory "
                         "(update: pinned or pageable buffer, H2D included)")
    ap.add_argument("--no-host-resident", action="store_true",
                    help="skip the H2D-inclusive sub-measurement of the default C2 line")
    ap.add_argument("--no-c4", action="store_true",
                    help="skip the BASELINE config-4 sub-measurement of multi-GPU runs")
    ap.add_argument("--no-c5", action="store_true",
                    help="skip the config-5 loopback upload sub-measurement of the default line")
    ap.add_argument("--no-configs", action="store_true",
                    help="skip the C3 / C4-shard sub-measurements of the default N=1 line")
    ap.add_argument("--print-launch", action="store_true",
                    help="--gpus N > 1 without a launcher: print the child launch command "
                         "and exit (tests)")
    ap.add_argument("--rank-dry-run", action="store_true",
                    help="tests: every rank joins the gloo group and rank 0 prints the ranks' "
                         "identities -- the launch path without any GPU call")
    return ap.parse_args(argv)


def launch_command(n: int, argv: list[str], port: int) -> tuple[list[str], dict]:
    """The child that runs `bench.py <argv>` as N ranks on one node: torch.distributed.run
    with one process per GPU and rendezvous on 127.0.0.1:port.  Returns (argv, env
    overrides); the child's ranks find WORLD_SIZE set and run the benchmark itself."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={n}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), *argv]
    # dmabuf IPC only on these hosts (a rank that shares device memory needs it), and the
    # launcher must not pick its own OMP thread count for the ranks' CPU work
    env = {"HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
           "OMP_NUM_THREADS": os.environ.get("OMP_NUM_THREADS", "1"),
           "S3H_BENCH_LAUNCHED": "1"}
    return cmd, env


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args, argv: list[str]) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher.  This process has made no GPU
    call (no torch.cuda, no s3h_*: torch is not even imported), so it may start the N ranks
    as ONE child process -- never an exec -- whose stdout (rank 0's JSON line) goes straight
    to ours; it exits with the child's return code."""
    import subprocess
    cmd, env = launch_command(args.gpus, argv, free_port())
    if args.print_launch:
        print(json.dumps({"cmd": cmd, "env": env, "torch_imported": "torch" in sys.modules}))
        return 0
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.run(cmd, env={**os.environ, **env}).returncode


def c3_length(p: int) -> int:
    z = ((SEED ^ 0xA5A5A5A5A5A5A5A5) ^ p) + 0x9E3779B97F4A7C15
    z &= (1 << 64) - 1
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & ((1 << 64) - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & ((1 << 64) - 1)
    z ^= z >> 31
    return 5 * MIB + z % (59 * MIB + 1)


def workload(cfg: str, rank: int, world: int, ppg: int, part_bytes: int = 0):
    """Global part ids, lengths and packed offsets of this rank's shard (s3client_amd.shard)."""
    from s3client_amd.shard import pack_offsets, shard_ids
    if cfg == "c3":
        n_total = ppg * world if ppg else 4096
        ids = shard_ids(n_total, rank, world)
        lens = np.array([c3_length(int(p)) for p in ids], dtype=np.uint64)
        name = f"C3: {n_total} parts x U[5,64] MiB (ragged)"
    else:
        per = ppg or (8192 if cfg == "c4" else 1024)
        ids = shard_ids(per * world, rank, world)
        pb = part_bytes or 8 * MIB
        lens = np.full(per, pb, dtype=np.uint64)
        name = (f"C2: 1024 parts x 8 MiB per GPU" if cfg == "c2" and not ppg and not part_bytes
                else f"{per} parts x {pb} B per GPU")
    return ids, lens, pack_offsets(lens), name


def isa_key(kname: str, nparts: int) -> str:
    """tools/isa_counts.py key of the kernel a plan runs (the two-group skew grid above 2,048)."""
    return "skew_nc2" if kname == "skew" and nparts > 2048 else kname


def library_info(keys=()) -> dict:
    """Which libs3hash.so this run loaded (S3H_LIBRARY may name an experiment build), its
    sha256, and the code hashes of the kernels measured (tools/code_object.py: the key that
    profiles/*_pmc.json records, so a counter profile is only used for the code it measured)."""
    from s3client_amd import _native
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import code_object
    import isa_counts
    path = _native.LIB_PATH
    info = {"path": os.path.relpath(path, ROOT), "sha256": code_object.file_sha256(path),
            "product_build": os.path.realpath(path) == os.path.realpath(
                os.path.join(ROOT, "s3client_amd", "lib", "libs3hash.so"))}
    try:
        lines = code_object.disassemble(path)
        info["kernel_code_hash"] = {k: code_object.code_hash(lines, isa_counts.ALL_KERNELS[k])
                                    for k in keys if k in isa_counts.ALL_KERNELS}
    except Exception as e:  # no llvm-objdump: the profile link is then unverifiable
        info["kernel_code_hash"] = {}
        info["kernel_code_hash_error"] = repr(e)
    return info


def pmc_traffic(cfg: str, kname: str, key: str, code_hash, algo_bytes: float):
    """HBM bytes per launch from the newest committed rocprofv3 --pmc summary of this config
    and kernel (profiles/rNN_<cfg>_<kernel>_pmc.json: FETCH_SIZE x2 + WRITE_SIZE, separate
    passes, tools/pmc_summary.py), scaled to this launch -- ONLY if that profile measured the
    same kernel machine code as this run loaded (its kernel_code_hash); otherwise null with
    the reason.  Returns (traffic, source, note)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{cfg}_{kname}_pmc.json")))
    if not files:
        return None, None, "no PMC profile of this config and kernel"
    rel = os.path.relpath(files[-1], ROOT)
    with open(files[-1]) as f:
        s = json.load(f)
    if not code_hash:
        return None, rel, "kernel code hash of this build unavailable: profile link unverifiable"
    if s.get("kernel_key") != key or s.get("kernel_code_hash") != code_hash:
        return None, rel, (f"{rel} measured kernel {s.get('kernel_key')} code "
                           f"{s.get('kernel_code_hash')}; this build runs {key} code {code_hash}")
    ratio = s["traffic_bytes_per_launch"] / s["algorithmic_bytes_per_launch"]
    return int(round(ratio * algo_bytes)), rel, (
        f"same kernel code {code_hash} (profile: library {str(s.get('library_sha256'))[:12]}, "
        f"commit {str(s.get('git_head'))[:12]})")


def clock_probe(torch, plan, info, data, digests, stream, dev, kname=None):
    """One extra launch (outside any timed region) on which every consumer wave of a skew /
    skewp / skews / MD5 plan records s_memtime and s_memrealtime around its chain loop -> the
    live shader clock and cycles per block; None for kernels without the probe."""
    if (kname or info["kernel"]) not in ("skew", "skewp", "skews", "md5-pc"):
        return None
    clocks = torch.zeros(4 * 4 * max(info["grid"], info["groups"]), dtype=torch.int64, device=dev)
    waves = plan.set_clock_probe(clocks)
    plan.launch(data, digests, stream)
    torch.cuda.synchronize(dev)
    plan.set_clock_probe(None)
    plan.status(stream)
    c = clocks.view(-1, 4)[:waves].cpu().numpy().astype(np.float64)
    cyc, rt = c[:, 1] - c[:, 0], c[:, 3] - c[:, 2]
    ok = rt > 0
    if not ok.any():
        return None
    return {"clock_GHz": round(float(np.median(cyc[ok] / rt[ok] * 0.1)), 3),  # rt: 100 MHz ticks
            "cycles_per_block": round(float(np.max(cyc[ok])) / info["max_blocks"], 1),
            "waves": int(ok.sum())}


def _cgroup_cpu_quota():
    """CPUs this container may use per the cgroup v2/v1 quota (None: unlimited/unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else round(int(q) / int(per), 2)
    except Exception:
        pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else round(q / per, 2)
    except Exception:
        return None


def _cpu_baseline_lib():
    """oracle/cpu_baseline.c (lib/hash's cost structure) built HERE with the reference's release
    flags -Ofast -march=native -flto (lib/CMakeLists.txt:45); the prebuilt portable
    oracle/libcpubase.so (-march=x86-64-v3) if no compiler is usable."""
    import tempfile
    src = os.path.join(ROOT, "oracle", "cpu_baseline.c")
    out = os.path.join(tempfile.mkdtemp(prefix="s3h_cpubase_"), "libcpubase_native.so")
    flags = "-Ofast -march=native -flto -DNDEBUG"
    try:
        import subprocess
        subprocess.run(["gcc", "-std=gnu11", *flags.split(), "-fPIC", "-shared", "-pthread",
                        "-o", out, src], check=True, capture_output=True, timeout=120)
        return out, flags
    except Exception:
        return os.path.join(ROOT, "oracle", "libcpubase.so"), "-Ofast -march=x86-64-v3 -flto (prebuilt)"


def cpu_baseline(host: np.ndarray, offs, lens, gpu_digests: np.ndarray, nsample: int,
                 algo: str = "sha256"):
    """lib/hash's sha256::sha256 cost structure (oracle/cpu_baseline.c, calibrated against the
    real lib/hash: profiles/r02_cpu_baseline_calibration.json) timed on this host's cores over
    the same parts as the GPU: one thread per available CPU (sched_getaffinity) and one per
    CPU of the cgroup quota, the faster of the two reported, parts round-robin, plus a
    1-thread figure.  MD5: the oracle port (the reference has no padded
    in-memory md5, md5.cpp:119-122)."""
    from tests.oracle_lib import ORACLE_SO, u64p
    if algo == "md5":
        path, flags = ORACLE_SO, "-O2 (oracle)"
        fn = ctypes.CDLL(path).oracle_md5_batch
    else:
        path, flags = _cpu_baseline_lib()
        fn = ctypes.CDLL(path).base_sha256_batch
    words = 4 if algo == "md5" else 8
    fn.argtypes = [ctypes.c_void_p, u64p, u64p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int]
    affinity = len(os.sched_getaffinity(0))
    quota = _cgroup_cpu_quota()
    n = min(nsample, len(lens))
    o = np.ascontiguousarray(offs[:n], dtype=np.uint64)
    ln = np.ascontiguousarray(lens[:n], dtype=np.uint64)
    # One thread per available CPU (sched_getaffinity); when a cgroup quota is smaller than
    # that (the GPU box: 16 CPUs of a 128-core host) the over-subscribed run is throttled and
    # noisy, so the quota's thread count is timed too and the faster run is the baseline.
    counts = [int(os.environ["S3H_CPU_THREADS"])] if "S3H_CPU_THREADS" in os.environ else \
        sorted({affinity, max(1, min(affinity, int(np.ceil(quota))))} if quota else {affinity})
    runs = {}
    for threads in counts:
        out = np.zeros((n, words), dtype=np.uint32)
        t0 = time.perf_counter()
        fn(host.ctypes.data, o.ctypes.data_as(u64p), ln.ctypes.data_as(u64p), n, out.ctypes.data, threads)
        runs[threads] = (time.perf_counter() - t0, out)
    threads = min(runs, key=lambda k: runs[k][0])
    dt, out = runs[threads]
    n1 = min(16, n)
    out1 = np.zeros((n1, words), dtype=np.uint32)
    t1 = time.perf_counter()
    fn(host.ctypes.data, o.ctypes.data_as(u64p), ln.ctypes.data_as(u64p), n1, out1.ctypes.data, 1)
    dt1 = time.perf_counter() - t1
    parity = bool(np.array_equal(out, gpu_digests[:n]) and np.array_equal(out1, gpu_digests[:n1]))
    cpu_model = ""
    try:
        with open("/proc/cpuinfo") as f:
            cpu_model = next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except Exception:
        pass
    gib = float(ln.sum()) / 2**30
    parity = parity and all(np.array_equal(r[1], gpu_digests[:n]) for r in runs.values())
    return {"value": round(gib / dt, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
            "sample": f"{n} of the bench's parts ({gib:.2f} GiB, the same bytes as the GPU) with "
                      f"{'oracle/cpu_baseline.c (lib/hash sha256::sha256 cost structure)' if algo == 'sha256' else 'the oracle MD5 port'}"
                      f" on {threads} threads, parts round-robin (faster of {sorted(runs)} threads: "
                      f"sched_getaffinity count and cgroup quota)",
            "GiBps_by_threads": {str(k): round(gib / v[0], 3) for k, v in sorted(runs.items())},
            "affinity_cpus": affinity,
            "build_flags": flags, "cgroup_cpu_quota": quota,
            "single_thread_GiBps": round(float(ln[:n1].sum()) / 2**30 / dt1, 3),
            "single_thread_sample": f"{n1} parts",
            "calibration": "restatement / real lib/hash = 0.93-1.01 (1 thread, -march=native, "
                           "profiles/r02_cpu_baseline_calibration.json)",
            "cpu_model": cpu_model, "digests_match_gpu": parity}


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(args, sys.argv[1:])  # parent: no GPU call has been made
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.rank_dry_run:
        return rank_dry_run(dist, world, rank, local)

    import s3client_amd as s3
    ph = Phases(rank)
    errors: list = []  # sub-measurements that failed (rank 0): the line says so, rc != 0
    if world != args.gpus and rank == 0:
        errors.append({"where": "launch", "error": f"--gpus {args.gpus} but WORLD_SIZE={world}"})
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    # One process per GPU.  S3H_BENCH_SHARE_GPU=1 (rehearsal on a 1-GPU box only) maps ranks
    # onto the visible devices modulo their count.  The timing collectives (barrier, max over
    # ranks, per-rank parity) use gloo on the host in every multi-process run: the data path
    # has no collective at all, so RCCL would buy nothing, and the one-GPU rehearsal then runs
    # exactly the code of a real N-GPU run.
    share = os.environ.get("S3H_BENCH_SHARE_GPU") == "1"
    if not share and local >= torch.cuda.device_count():
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} "
                         "visible GPU(s): one process per GPU (S3H_BENCH_SHARE_GPU=1 to rehearse "
                         "several ranks on one GPU)")
    gpu = local % torch.cuda.device_count() if share else local
    torch.cuda.set_device(gpu)
    if world > 1:
        init_gloo(dist)
    dev = torch.device("cuda", gpu)
    local = gpu
    devices = gather_obj(dist, world, device_identity(torch, s3, gpu, rank))
    distinct = len({d["pci_bus_id"] for d in devices})
    if rank == 0 and distinct != world and not share:
        errors.append({"where": "devices", "error": f"{world} ranks ran on {distinct} distinct "
                                                    "devices (S3H_BENCH_SHARE_GPU unset)"})
    ph.mark("init")

    ids, lens, offs, name = workload(args.config, rank, world, args.parts_per_gpu,
                                    args.part_bytes)
    nbytes = int(offs[-1] + lens[-1]) + 256
    data = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, ids, SEED)
    stream = torch.cuda.current_stream(dev)
    plan = s3.Plan(offs, lens, device=local, kernel=args.kernel, algo=args.algo)
    digests = torch.zeros((len(lens), plan.words), dtype=torch.int32, device=dev)
    info = plan.info()
    kname = "md5-pc" if args.algo == "md5" else info["kernel"]

    if args.mode in ("host", "host-dual"):
        return host_mode(args, s3, torch, dist, data, ids, lens, offs, world, rank, name)
    if args.mode == "stream":
        return stream_mode(args, s3, torch, data, ids, lens, offs, rank, name, stream)
    if args.mode == "dual":
        return dual_mode(args, s3, torch, data, ids, lens, offs, rank, name, stream)

    for _ in range(args.warmup):
        plan.launch(data, digests, stream)
    torch.cuda.synchronize(dev)
    status_all(dist, world, lambda: plan.status(stream))
    ph.mark("setup+warmup")

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    with power_sampler(devices[rank]) as pw:
        t0 = time.perf_counter()
        for i in range(args.steps):
            ev[i][0].record(stream)
            plan.launch(data, digests, stream)
            ev[i][1].record(stream)
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        wall = time.perf_counter() - t0
    # every timed launch's device error word (a timed-out producer/consumer wait), gathered
    # from every rank before any rank raises (no rank is left waiting in a collective)
    status_all(dist, world, lambda: plan.status(stream))
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    t = torch.tensor([wall, kern_ms], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # max over ranks: the slowest GPU sets the time
    wall, kern_ms_max = float(t[0]), float(t[1])
    ph.mark(f"timed {args.steps} steps")

    probe = clock_probe(torch, plan, info, data, digests, stream, dev, kname)
    power = gather_obj(dist, world, pw.summary())

    # parity of the last timed step's digests against the reference fixtures, on EVERY rank
    # (tests/golden: C2/C4 parts and four parts of each rank's shard at N = 2, 4, 8)
    gd = digests.cpu().numpy().view(np.uint32)
    fixtures = golden_fixtures(args.config, args.algo, args.part_bytes)
    checked = bad = 0
    for slot, p in enumerate(ids):
        want = fixtures.get(int(p))
        if want is not None:
            checked += 1
            bad += s3.hash_to_text(gd[slot]) != want
    par = per_rank(dist, world, [checked, int(bad)])

    key = isa_key(kname, len(lens))
    lib_info = library_info([key])
    part_bytes = float(lens.sum())
    total_bytes = part_bytes * world * args.steps
    value = total_bytes / 2**30 / wall
    algo_bytes = part_bytes + 4 * plan.words * len(lens)  # read once + digests written
    achieved = algo_bytes / (kern_ms / 1e3) / 1e9      # GB/s, this rank's kernel
    compressions = info["total_blocks"]
    traffic, traffic_src, traffic_note = pmc_traffic(args.config, kname, key,
                                                     lib_info["kernel_code_hash"].get(key),
                                                     algo_bytes)
    # one part = one sequential chain on one lane: report what one chain sustains and how
    # many of the chip's 256 CU x 4 SIMD x 64 = 65,536 lanes the batch can occupy
    chain_gbps = float(lens.max()) / (kern_ms / 1e3) / 1e9
    issue = issue_model(kname, len(lens), kern_ms, info, probe)
    ph.mark("parity+probe")

    line = None
    if rank == 0:
        line = {
            "metric": ("device-resident SHA-256 GiB/s over 8 MiB parts; bit-exact digests vs lib/hash"
                       if args.algo == "sha256" else
                       "device-resident MD5 GiB/s over 8 MiB parts (SURVEY 8(f); not the metric)"),
            "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: generator G(seed=20241008) written in HBM by a HIP kernel",
            "config": {"workload": name, "parts_per_gpu": int(len(lens)),
                       "part_bytes": int(lens[0]) if args.config != "c3" else "5-64 MiB",
                       "kernel": kname, "grid": info["grid"], "groups": info["groups"],
                       "solo_workgroups": info["solo"],
                       "parallelism": f"parts sharded round-robin over {world} GPU(s), no collective"},
            "devices": devices, "distinct_devices": distinct,
            "parity": {"fixtures_checked": sum(r[0] for r in par),
                       "mismatches": sum(r[1] for r in par),
                       "per_rank": [{"rank": k, "fixtures_checked": r[0], "mismatches": r[1]}
                                    for k, r in enumerate(par)]},
            "status": "ok: device error word clear after every launch on every rank (s3h_plan_status)",
            "library": lib_info,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "traffic_source": traffic_src,
                         "traffic_note": traffic_note,
                         "kernel_ms": round(kern_ms, 3),
                         "kernel_ms_max_rank": round(kern_ms_max, 3),
                         "bytes_per_launch": int(algo_bytes),
                         "compressions_per_launch": int(compressions),
                         "compressions_per_s": round(compressions / (kern_ms / 1e3), 1),
                         "per_chain_GBps": round(chain_gbps, 4),
                         "lanes_occupied_frac": round(min(len(lens), 65536) / 65536, 5)},
            "issue": issue,
            "power": power[0] if world == 1 else power,
        }
        if world == 1:
            line["power"].update(energy(power[0], value))
        default_c2 = (world == 1 and args.config == "c2" and args.algo == "sha256"
                      and not args.parts_per_gpu and not args.part_bytes)
        if default_c2 and not args.no_host_resident:
            line["host_resident"] = _guard(errors, "host_resident", host_resident, s3, torch,
                                           data, ids, lens, offs, gd)
            ph.mark("host_resident")
            if not args.no_c5:
                line["c5_loopback"] = _guard(errors, "c5_loopback", c5_loopback, data, offs,
                                             lens, gd)
                ph.mark("c5_loopback")
        if default_c2 and not args.no_configs:
            line["f_rows"] = _guard(errors, "f_rows", f_rows_c2, s3, torch, data, ids, lens,
                                    offs, dev, stream)
            ph.mark("f_rows")
        if world == 1 and not args.no_cpu_baseline:
            n = min(args.cpu_sample_parts, len(lens))
            end = int(offs[n - 1] + lens[n - 1])
            host = data[:end].cpu().numpy()
            line["cpu_baseline"] = _guard(errors, "cpu_baseline", cpu_baseline, host, offs,
                                          lens, gd, n, args.algo)
            del host
            ph.mark("cpu_baseline")
        if default_c2 and not args.no_configs:
            del data, digests
            plan.close()
            torch.cuda.empty_cache()
            line["configs"] = {}
            for c in ("c3", "c4"):
                line["configs"][c] = _guard(errors, f"configs.{c}", single_gpu_config, s3,
                                            torch, dev, c, devices[0])
                ph.mark(f"configs.{c}")
    if world > 1 and args.config == "c2" and args.algo == "sha256":
        del data, digests
        plan.close()
        torch.cuda.empty_cache()
        if not args.no_c4:
            try:  # a device fault raises on EVERY rank together (status_all), so all catch it
                c4 = c4_shard(args, s3, torch, dist, dev, rank, world, local, devices[rank], ph)
            except DeviceFault as e:
                c4 = {"error": str(e)}
                if rank == 0:
                    errors.append({"where": "c4", "error": str(e), "device_fault": True})
            if rank == 0:
                line["c4"] = c4
        if not args.no_host_resident:
            dist.barrier()  # the other ranks wait while rank 0 drives every GPU from the host
            if rank == 0:
                line["host_resident"] = _guard(errors, "host_resident", host_resident_multi,
                                               s3, torch, dev, world, ph)
                ph.mark("host_resident (N devices)")
            dist.barrier()
    rc = 0
    if rank == 0:
        errors += parity_failures(line)
        line["phases_s"] = ph.times
        if errors:
            line["errors"] = errors
            rc = 3
        print(json.dumps(line), flush=True)
    if world > 1:
        rc = max(x[0] for x in per_rank(dist, world, [rc]))
        dist.destroy_process_group()
    return rc


def rank_dry_run(dist, world: int, rank: int, local: int) -> int:
    """--rank-dry-run: the multi-rank plumbing of a bench run (gloo group, gathered per-rank
    records, one line from rank 0, exit code agreed over ranks) with no GPU call, so the
    self-launch is testable on a CPU-only host."""
    import socket
    if world > 1:
        init_gloo(dist)
    me = {"rank": rank, "local_rank": local, "pid": os.getpid(), "host": socket.gethostname(),
          "launched_by_bench": os.environ.get("S3H_BENCH_LAUNCHED") == "1"}
    ranks = gather_obj(dist, world, me)
    if rank == 0:
        print(json.dumps({"n_gpus": world, "ranks": ranks}), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


class DeviceFault(RuntimeError):
    """A device error word (or another status check) failed on at least one rank."""


class Phases:
    """Seconds per phase of this rank's run, to stderr as they end (rank 0) and into the line:
    an N-GPU line's time is accounted for against the driver's clock."""

    def __init__(self, rank: int):
        self.rank, self.t, self.times = rank, time.perf_counter(), {}

    def mark(self, name: str) -> None:
        now = time.perf_counter()
        self.times[name] = round(now - self.t, 3)
        if self.rank == 0:
            print(f"[bench rank 0] {name}: {now - self.t:.2f} s", file=sys.stderr, flush=True)
        self.t = now


def device_identity(torch, s3, gpu: int, rank: int) -> dict:
    """Which physical GPU this rank hashed on: the PCI address as libs3hash's own HIP context
    reports it (s3h_device_pci_bus_id), the name and UUID torch reports, host and pid."""
    import socket
    p = torch.cuda.get_device_properties(gpu)
    return {"rank": rank, "device_index": gpu, "pci_bus_id": s3.device_pci_bus_id(gpu),
            "torch_pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "name": p.name, "arch": getattr(p, "gcnArchName", ""), "uuid": str(p.uuid),
            "cus": p.multi_processor_count, "host": socket.gethostname(), "pid": os.getpid()}


def gather_obj(dist, world: int, obj):
    """[obj of rank 0, obj of rank 1, ...] over gloo; [obj] at N = 1."""
    if world == 1:
        return [obj]
    out = [None] * world
    dist.all_gather_object(out, obj)
    return out


def status_all(dist, world: int, check) -> None:
    """Run a status check (plan.status: the device error word) on every rank and gather every
    rank's outcome BEFORE raising, so a fault on one rank fails all of them together instead
    of leaving the others blocked in the next collective."""
    err = ""
    try:
        check()
    except Exception as e:  # noqa: BLE001 -- re-raised on every rank below
        err = f"{type(e).__name__}: {e}"
    bad = [(k, e) for k, e in enumerate(gather_obj(dist, world, err)) if e]
    if bad:
        raise DeviceFault("; ".join(f"rank {k}: {e}" for k, e in bad))


def power_sampler(ident: dict):
    """Board power + GFX clock of this rank's device over a timed region (tools/power.py)."""
    tools = os.path.join(ROOT, "tools")
    if tools not in sys.path:
        sys.path.insert(0, tools)
    from power import PowerSampler
    return PowerSampler(ident["pci_bus_id"])


def issue_model(kname: str, nparts: int, kern_ms: float, info: dict, probe) -> dict:
    """Per-wave issue roof of the chain loop: cycles per block (clock probe, else kernel time x
    the assumed clock) over the instructions per block read from the shipped code object."""
    if probe:
        cyc_per_block, clock_src = probe["cycles_per_block"], "in-kernel s_memtime probe"
    else:
        cyc_per_block = kern_ms / 1e3 * CLOCK_GHZ * 1e9 / info["max_blocks"]
        clock_src = f"kernel time x assumed {CLOCK_GHZ} GHz"
    ipb, ipb_src = chain_instr_per_block(kname, 2 if (kname == "skew" and nparts > 2048) else 1)
    cpi = cyc_per_block / ipb
    return {"bound": "per-wave instruction issue of each part's sequential chain",
            "chain_instr_per_block": ipb, "chain_instr_source": ipb_src,
            "cycles_per_block": round(cyc_per_block, 1), "cycles_source": clock_src,
            "cycles_per_instr": round(cpi, 3),
            # floor: one wave issues at most one instruction per 4 cycles (MI355X_MICROARCH.md
            # 'vector-instruction ISSUE cost'; 4.05 measured on an aligned lone-wave stream,
            # profiles/r01_ubench_alignment.txt)
            "issue_floor_cycles_per_instr": ISSUE_FLOOR_CPI,
            "frac": round(ISSUE_FLOOR_CPI / cpi, 4),
            "clock_GHz": probe["clock_GHz"] if probe else CLOCK_GHZ,
            # chip-wide INT32-VALU roof (256 CU x 64 lanes x clock / VALU per
            # block of the one-lane-per-part kernel x 64 B) and the parallelism ceiling
            "valu_roof_GBps": round(256 * 64 * CLOCK_GHZ * 1e9 / HAND_INSTR_PER_BLOCK["lane"]
                                    * 64 / 1e9, 1),
            "parallelism_ceiling": round(min(nparts, 65536) / 65536, 5)}


def energy(power: dict, gibps: float) -> dict:
    """Joules per GiB hashed (board power over the timed launches / rate) and the energy-delay
    product (J/GiB x s/GiB) that s3h_kernel_policy's "efficiency" minimises."""
    w = power.get("busy_mean_W") if isinstance(power, dict) else None
    if not w or not gibps:
        return {}
    return {"J_per_GiB": round(w / gibps, 4),
            "energy_delay_J_s_per_GiB2": round(w / gibps / gibps, 7)}


def parity_failures(obj, path: str = "") -> list:
    """Every digest comparison in the line that failed: a non-zero mismatch count or a false
    digests-match flag anywhere in the nested sub-measurements."""
    out = []
    if isinstance(obj, dict):
        for k, v in obj.items():
            p = f"{path}.{k}" if path else k
            if k in ("mismatches", "fixture_mismatches") and isinstance(v, int) and v > 0:
                out.append({"where": p, "error": f"{v} digest mismatches"})
            elif (k.startswith("digests_match") or k.endswith("_equals_sha256_only_run")) and v is False:
                out.append({"where": p, "error": "digests differ"})
            elif isinstance(v, (dict, list)):
                out += parity_failures(v, p)
    elif isinstance(obj, list):
        for i, v in enumerate(obj):
            out += parity_failures(v, f"{path}[{i}]")
    return out


def _guard(errors: list, where: str, fn, *args):
    """A sub-measurement of the line (rank 0, after the timed region and its parity): an
    exception is reported in its place AND in the line's top-level `errors` (the process then
    exits non-zero) instead of losing the metric line."""
    try:
        return fn(*args)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        import traceback
        traceback.print_exc(file=sys.stderr)
        from s3client_amd import S3HashError
        msg = f"{type(e).__name__}: {e}"
        errors.append({"where": where, "error": msg, "device_fault": isinstance(e, S3HashError)})
        return {"error": msg}


def init_gloo(dist) -> None:
    """init_process_group("gloo") with the process's stdout pointed at stderr meanwhile: gloo
    prints "[Gloo] Rank r is connected to ..." on stdout (fd 1, from C++) in every rank, and
    the bench's stdout must hold exactly one line -- rank 0's JSON."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group("gloo")
    finally:
        os.dup2(saved, 1)
        os.close(saved)


def per_rank(dist, world: int, vals):
    """[vals of rank 0, vals of rank 1, ...] (int64) -- gloo all_gather; [vals] at N = 1."""
    import torch
    t = torch.tensor(vals, dtype=torch.int64)
    if world == 1:
        return [[int(x) for x in t]]
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    return [[int(x) for x in a] for a in allt]


def h2d_copy_rate(torch, host, dev, chunk: int = 1 << 30, reps: int = 3,
                  rows: int = 0, row_bytes: int = 0) -> dict:
    """The roof of the host-resident path: a plain pinned -> HBM copy of the same pinned bytes
    (1 GiB hipMemcpyAsync chunks back to back into one device buffer, no hashing), best of
    ``reps`` passes, timed with HIP events on the copy stream.  With ``rows``: also the same
    bytes as the host path moves them -- one hipMemcpy2DAsync per slice of ``row_bytes`` from
    each of ``rows`` parts at the parts' pitch -- so the two copy shapes can be told apart."""
    n = host.numel()
    s = torch.cuda.current_stream(dev)

    def best_of(body, dst):
        best = None
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            body(dst)
            b.record(s)
            torch.cuda.synchronize(dev)
            ms = a.elapsed_time(b)
            best = ms if best is None else min(best, ms)
        return round(n / 2**30 / (best / 1e3), 3)

    def flat(dst):
        for o in range(0, n, chunk):
            m = min(chunk, n - o)
            dst[:m].copy_(host[o:o + m], non_blocking=True)

    dst = torch.empty(min(chunk, n), dtype=torch.uint8, device=dev)
    res = {"GiBps": best_of(flat, dst), "bytes": n, "chunk_bytes": chunk,
           "what": "pinned host -> HBM copy of the same bytes, no hashing (best of %d)" % reps}
    del dst
    if rows and row_bytes and n % rows == 0 and (n // rows) % row_bytes == 0:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy2DAsync.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
                                         ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_int, ctypes.c_void_p]
        pitch = n // rows
        dst = torch.empty(rows * row_bytes, dtype=torch.uint8, device=dev)
        src0, sh = host.data_ptr(), ctypes.c_void_p(s.cuda_stream)

        def two_d(d):
            for k in range(pitch // row_bytes):
                rc = hip.hipMemcpy2DAsync(d.data_ptr(), row_bytes, src0 + k * row_bytes, pitch,
                                          row_bytes, rows, 1, sh)  # 1 = hipMemcpyHostToDevice
                if rc:
                    raise RuntimeError(f"hipMemcpy2DAsync failed: {rc}")

        res["GiBps_2d_slices"] = best_of(two_d, dst)
        res["slice"] = f"{rows} rows x {row_bytes} B at a {pitch} B pitch"
        del dst
    return res


def allowed_mem_nodes() -> list:
    """NUMA nodes this process may allocate on (/proc/self/status Mems_allowed_list)."""
    try:
        with open("/proc/self/status") as f:
            s = next(l.split(":", 1)[1].strip() for l in f if l.startswith("Mems_allowed_list"))
    except (OSError, StopIteration):
        return []
    out = []
    for part in s.split(","):
        lo, _, hi = part.partition("-")
        out += list(range(int(lo), int(hi or lo) + 1))
    return out


def pinned_on(s3, torch, nbytes: int, node: int):
    """(PinnedBuffer on NUMA node `node`, CPU torch view of it)."""
    buf = s3.PinnedBuffer(nbytes, node)
    return buf, torch.from_numpy(buf.array)


def host_resident(s3, torch, data, ids, lens, offs, gd, reps: int = 3):
    """The same C2 batch starting and ending in HOST memory (H2D included): the parts are
    copied once into pinned memory on the device's NUMA node (s3h_host_alloc, outside the timed
    region), then s3h_sha256_batch_host streams them through the HBM ring and returns the
    digests to the host.  On a multi-node host the same bytes are also pinned on another node
    and the two buffers timed alternately (`numa`: the local/remote A/B)."""
    end = int(offs[-1] + lens[-1])
    dev = data.device
    dev_node = s3.device_numa(dev.index)["node"]
    local_buf, host = pinned_on(s3, torch, end, dev_node)
    host.copy_(data[:end])
    parts = s3.BufferParts(host, offs, lens)  # part pointers formed in numpy
    out = s3.sha256_batch_host(parts, ndevices=1)  # warm: the per-device context is cached
    gib = float(lens.sum()) / 2**30

    def timed(p):
        t0 = time.perf_counter()
        o = s3.sha256_batch_host(p, ndevices=1)
        return time.perf_counter() - t0, o

    others = [n for n in allowed_mem_nodes() if n != dev_node] if dev_node >= 0 else []
    remote = rparts = rhost = None
    if others:
        remote, rhost = pinned_on(s3, torch, end, others[0])
        rhost.copy_(host)
        rparts = s3.BufferParts(rhost, offs, lens)
        s3.sha256_batch_host(rparts, ndevices=1)
    times, rtimes, rsame = [], [], True
    for _ in range(reps):  # local and remote alternately
        t, out = timed(parts)
        times.append(t)
        if rparts is not None:
            t, ro = timed(rparts)
            rtimes.append(t)
            rsame = rsame and bool(np.array_equal(ro, out))
    uniform = bool((np.diff(offs) == lens[0]).all() and (lens == lens[0]).all()) and offs[0] == 0
    h2d = h2d_copy_rate(torch, host, dev, rows=len(lens) if uniform else 0,
                        row_bytes=256 * 1024)
    numa = {"device_node": dev_node, "buffer_node": s3.mem_node(host),
            "host_path": s3.host_numa_info(dev.index),
            "policy": "staging + copy threads on the device's node (s3h_host_numa local)"}
    if rparts is not None:
        rh2d = h2d_copy_rate(torch, rhost, dev)
        numa.update({"remote_buffer_node": s3.mem_node(rhost),
                     "local_GiBps": round(gib / float(np.mean(times)), 3),
                     "remote_GiBps": round(gib / float(np.mean(rtimes)), 3),
                     "remote_over_local": round(float(np.mean(times)) / float(np.mean(rtimes)), 4),
                     "remote_h2d_copy_GiBps": rh2d["GiBps"],
                     "digests_match_remote_run": rsame,
                     "ab": f"{reps} alternating calls per buffer, same bytes pinned on node "
                           f"{dev_node} (local) and node {others[0]} (remote)"})
    res = {"metric": "host-resident (H2D-inclusive) SHA-256 GiB/s, same C2 parts",
           "value": round(gib / float(np.mean(times)), 3), "best": round(gib / min(times), 3),
           "unit": "GiB/s", "ms_per_batch": round(1e3 * float(np.mean(times)), 2), "reps": reps,
           "h2d_copy": h2d,
           "frac_of_h2d_copy": round(gib / float(np.mean(times)) / h2d["GiBps"], 4),
           "numa": numa,
           "path": "pinned host parts (device's NUMA node) -> 3-slot HBM ring (one 2-D H2D copy "
                   "per 256 KiB slice) -> skew kernel per slice -> digests D2H "
                   "(s3h_sha256_batch_host)",
           "fixture_mismatches": _fixture_mismatches(s3, ids, out),
           "digests_match_device_run": bool(np.array_equal(out, gd))}
    res["split"] = split_from_host(s3, parts, lens, gd)
    res["stream"] = stream_from_host(s3, host, offs, lens, gd)
    del host, parts, rhost, rparts, local_buf, remote
    return res


def split_from_host(s3, parts, lens, gd, reps: int = 3) -> dict:
    """The same pinned C2 parts on S3H_ROUTE_SPLIT: the CPU drop-in (SHA-NI on the host
    threads) hashes the model's share of the parts while the GPU host path hashes the rest, at
    once -- the upload path's rate when the host's cores help; NOT a GPU-only number (`value`
    above is).  What AUTO takes for this batch is reported beside it."""
    gib = float(lens.sum()) / 2**30
    s3.sha256_batch_routed(parts, ndevices=1, route="split")  # warm
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out, taken = s3.sha256_batch_routed(parts, ndevices=1, route="split")
        times.append(time.perf_counter() - t0)
    model = s3.route_model()
    k, _, est = s3.route_split_estimate(lens, model, ndevices=1)
    auto_out, auto_taken = s3.sha256_batch_routed(parts, ndevices=1, route="auto")
    return {"metric": "host-resident SHA-256 GiB/s, GPU host path and CPU drop-in at once (S3H_ROUTE_SPLIT)",
            "GiBps": round(gib / float(np.mean(times)), 3), "ms_per_batch": round(1e3 * float(np.mean(times)), 2),
            "reps": reps, "taken": taken, "cpu_parts": k, "gpu_parts": int(len(lens) - k),
            "cpu_threads": model["cpu_threads"], "cpu_backend": s3.cpu_backend(),
            "model_s": round(est, 4), "auto_takes": auto_taken,
            "digests_match_device_run": bool(np.array_equal(out, gd) and np.array_equal(auto_out, gd))}


def stream_from_host(s3, host, offs, lens, gd, chunk: int = MIB, reps: int = 2) -> dict:
    """SURVEY 8(f).2 on the same pinned bytes: the C2 parts as len(lens) streamed objects
    appended in `chunk`-byte pieces from host memory (s3h_stream_update_host: each update's copy
    overlaps the previous update's hash) and finished; one object reused across passes (final()
    restarts it).  Wall time per pass; digests vs the device run."""
    n = len(lens)
    nupd = int((int(lens.max()) + chunk - 1) // chunk)
    gib = float(lens.sum()) / 2**30

    def one_pass(st):
        for k in range(nupd):
            lk = np.minimum(np.maximum(lens.astype(np.int64) - k * chunk, 0), chunk).astype(np.uint64)
            st.update(s3.BufferParts(host, offs + np.uint64(k * chunk), lk))
        return st.final()

    with s3.Stream(n) as st:
        out = one_pass(st)  # warm: staging sets and pieces
        times = []
        for _ in range(reps):
            t0 = time.perf_counter()
            out = one_pass(st)
            times.append(time.perf_counter() - t0)
    return {"metric": "streamed-object SHA-256 GiB/s from pinned host memory (H2D included)",
            "GiBps": round(gib / float(np.mean(times)), 3), "objects": n, "chunk_bytes": chunk,
            "updates_per_pass": nupd, "reps": reps,
            "digests_match_device_run": bool(np.array_equal(out, gd))}


def f_rows_c2(s3, torch, data, ids, lens, offs, dev, stream, steps: int = 3) -> dict:
    """SURVEY 8(f) kernels on the C2 parts already resident, so the driver's default run also
    records them: Content-MD5 alone (md5_pc_kernel, HIP-event kernel time) and both upload
    digests from one pass (s3h_sha256_md5_batch_device, wall time per call incl. its sync),
    each with fixture parity (lib/hash SHA-256 and md5_file goldens)."""
    gib = float(lens.sum()) / 2**30
    plan = s3.Plan(offs, lens, device=dev.index, algo="md5")
    out = torch.zeros((len(lens), plan.words), dtype=torch.int32, device=dev)
    plan.launch(data, out, stream)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(steps)]
    for a, b in ev:
        a.record(stream)
        plan.launch(data, out, stream)
        b.record(stream)
    torch.cuda.synchronize(dev)
    plan.status(stream)  # device error word clear (raises otherwise)
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    m5 = out.cpu().numpy().view(np.uint32)
    mf = golden_fixtures("c2", "md5")
    chk = [k for k, p in enumerate(ids) if int(p) in mf]
    bad = sum(s3.digests_to_text(m5[k:k + 1], 4)[0] != mf[int(ids[k])] for k in chk)
    plan.close()
    res = {"md5": {"metric": "device-resident MD5 GiB/s (Content-MD5), C2 parts",
                   "kernel": "md5-pc", "GiBps": round(gib / (kern_ms / 1e3), 3),
                   "kernel_ms": round(kern_ms, 3), "steps": steps,
                   "parity": {"fixtures_checked": len(chk), "mismatches": int(bad)}}}
    del out
    sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
        times.append(time.perf_counter() - t0)
    bad = _fixture_mismatches(s3, ids, sha.cpu().numpy().view(np.uint32), m5.cpu().numpy().view(np.uint32))
    wall = float(np.mean(times))
    res["sha256_md5"] = {"metric": "device-resident SHA-256 + MD5 GiB/s (both digests, one pass), "
                                   "C2 parts", "GiBps": round(gib / wall, 3),
                         "ms_per_call": round(wall * 1e3, 3), "steps": steps,
                         "fixture_mismatches": int(bad)}
    del sha, m5
    return res


def single_gpu_config(s3, torch, dev, cfg: str, ident: dict, steps: int = 2) -> dict:
    """BASELINE configs 3 and 4 beside the C2 headline of the default N=1 line, so every
    single-GPU configuration has a driver-run number: C3 = 4,096 x U[5,64] MiB (~138 GiB
    resident), C4 = rank 0's shard of 65,536 x 8 MiB over 8 GPUs (parts 8k, 64 GiB).  Each
    kernel timed with HIP events on the launch stream, then the in-kernel clock probe (live
    shader clock, cycles per block -> fraction of the issue floor) and the board power over the
    timed launches (amdsmi), fixture parity.  C3: AUTO.  C4: AUTO (skews, shared-SIMD
    producers) AND skewp beside it, so the line itself shows what the C4 kernel choice buys and
    at what power."""
    from s3client_amd.shard import pack_offsets, shard_ids
    if cfg == "c3":
        ids, lens, offs, name = workload("c3", 0, 1, 0)
    else:
        ids = shard_ids(65536, 0, 8)
        lens = np.full(8192, 8 * MIB, dtype=np.uint64)
        offs = pack_offsets(lens)
        name = "C4: rank 0 of 8 -- 8192 x 8 MiB (global parts 8k)"
    data = torch.empty(int(offs[-1] + lens[-1]) + 256, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, ids, SEED)
    stream = torch.cuda.current_stream(dev)
    fx = golden_fixtures(cfg, "sha256")
    part_bytes = float(lens.sum())
    algo = part_bytes + 32 * len(lens)
    kernels = {}
    gd = info = None
    # C4 times both kernels AUTO chooses between (by s3h_kernel_policy) explicitly, so the line
    # carries skews and skewp whichever the default policy picks on this board
    with s3.Plan(offs, lens, device=dev.index) as p:
        info = p.info()
    for kern in (("auto",) if cfg == "c3" else ("skews", "skewp")):
        plan = s3.Plan(offs, lens, device=dev.index, kernel=kern)
        kinfo = plan.info()
        out = torch.zeros((len(lens), 8), dtype=torch.int32, device=dev)
        plan.launch(data, out, stream)
        torch.cuda.synchronize(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        with power_sampler(ident) as pw:
            t0 = time.perf_counter()
            for a, b in ev:
                a.record(stream)
                plan.launch(data, out, stream)
                b.record(stream)
            torch.cuda.synchronize(dev)
            wall = (time.perf_counter() - t0) / steps
        plan.status(stream)  # device error word clear (raises otherwise)
        kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
        probe = clock_probe(torch, plan, kinfo, data, out, stream, dev)
        kd = out.cpu().numpy().view(np.uint32)
        checked = [k for k, p in enumerate(ids) if int(p) in fx]
        bad = sum(s3_hex(kd[k]) != fx[int(ids[k])] for k in checked)
        plan.close()
        del out
        iss = issue_model(kinfo["kernel"], len(lens), kern_ms, kinfo, probe)
        kernels[kinfo["kernel"]] = {
            "GiBps": round(part_bytes / 2**30 / wall, 3), "ms_per_step": round(1e3 * wall, 3),
            "kernel_ms": round(kern_ms, 3), "grid": kinfo["grid"],
            "hbm_roofline_frac": round(algo / (kern_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 5),
            "clock_GHz": probe["clock_GHz"] if probe else None,
            "cycles_per_block": probe["cycles_per_block"] if probe else None,
            "chain_instr_per_block": iss["chain_instr_per_block"],
            "issue_frac": iss["frac"] if probe else None,
            "power": pw.summary(),
            "parity": {"fixtures_checked": len(checked), "mismatches": int(bad)}}
        kernels[kinfo["kernel"]].update(energy(kernels[kinfo["kernel"]]["power"],
                                               part_bytes / 2**30 / wall))
        if gd is None:
            gd = kd
            if kern == "auto":
                info = kinfo
        elif not np.array_equal(kd, gd):
            kernels[kinfo["kernel"]]["digests_match_other_kernel"] = False
        if kinfo["kernel"] == info["kernel"]:
            auto_digests = kd
    gd = auto_digests
    dual = _dual_on(s3, torch, dev, data, ids, lens, offs, cfg, stream, gd, info) if cfg == "c3" else None
    del data
    torch.cuda.empty_cache()
    auto = kernels[info["kernel"]]
    res = {"workload": name, "kernel": info["kernel"], "grid": info["grid"],
           "solo_workgroups": info["solo"], "steps": steps,
           **{k: auto[k] for k in ("GiBps", "ms_per_step", "kernel_ms", "hbm_roofline_frac",
                                   "clock_GHz", "cycles_per_block", "issue_frac", "power")},
           "bound": "the longest part's chain" if cfg == "c3" else "per-wave issue of 8,192 chains",
           "parity": auto["parity"]}
    res.update(energy(auto["power"], auto["GiBps"]))
    if len(kernels) > 1:
        res["kernels"] = kernels
        # s3h_kernel_policy: AUTO under "throughput" = the faster kernel, under "efficiency"
        # = the lower energy-delay product (J/GiB x s/GiB), under "power" (the default) skews
        # only when the board's power cap lets it hold its clock
        ok = {k: v for k, v in kernels.items() if v.get("energy_delay_J_s_per_GiB2")}
        chosen = {}
        for pol in ("throughput", "efficiency", "power"):
            prev = s3.kernel_policy(pol)
            try:
                with s3.Plan(offs, lens, device=dev.index) as p:
                    chosen[pol] = p.info()["kernel"]
            finally:
                s3.kernel_policy(prev)
        res["policy_choice"] = {
            "measured_faster": max(kernels, key=lambda k: kernels[k]["GiBps"]),
            "measured_lower_energy_delay": min(
                ok, key=lambda k: ok[k]["energy_delay_J_s_per_GiB2"]) if ok else None,
            "board_power_cap_W": s3.device_power_cap(dev.index),
            **{f"auto_{pol}_policy": k for pol, k in chosen.items()}}
    if dual:
        res["sha256_md5"] = dual
    return res


def _dual_on(s3, torch, dev, data, ids, lens, offs, cfg, stream, gd, info, steps: int = 2) -> dict:
    """SHA-256 + MD5 of the same resident parts in one pass (s3h_sha256_md5_batch_device: for
    C3 the mixed grid, info["dual_solo"] skew workgroups), wall time per call incl. its sync;
    SHA-256 digests must equal the SHA-256-only run's, MD5 checked against the lib/hash
    md5_file fixtures."""
    sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
    torch.cuda.synchronize(dev)
    times = []
    for _ in range(steps):
        t0 = time.perf_counter()
        sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
        times.append(time.perf_counter() - t0)
    wall = float(np.mean(times))
    same = bool(np.array_equal(sha.cpu().numpy().view(np.uint32), gd))
    mf = golden_fixtures(cfg, "md5")
    m5h = m5.cpu().numpy().view(np.uint32)
    chk = [k for k, p in enumerate(ids) if int(p) in mf]
    bad = sum(s3.digests_to_text(m5h[k:k + 1], 4)[0] != mf[int(ids[k])] for k in chk)
    del sha, m5
    return {"metric": "device-resident SHA-256 + MD5 GiB/s (both digests, one pass)",
            "GiBps": round(float(lens.sum()) / 2**30 / wall, 3), "ms_per_call": round(wall * 1e3, 2),
            "steps": steps, "dual_solo_workgroups": info.get("dual_solo", 0),
            "sha256_equals_sha256_only_run": same,
            "md5_parity": {"fixtures_checked": len(chk), "mismatches": int(bad)}}


def c5_loopback(data, offs, lens, gd, nparts: int = 128, jobs: int = 16, repeat: int = 2):
    """BASELINE config 5 without MinIO (absent here): C2 parts 0..nparts-1 written to a file,
    which apps/s3_upload_hash slices as `jobs` x nparts/jobs parts (upload.cpp geometry: the
    same 8 MiB parts) and uploads as the reference's UploadFile does (upload.cpp:113-149,
    `--multipart`): CreateMultipartUpload, every part hashed and PUT with its digest signed
    into x-amz-content-sha256, CompleteMultipartUpload with the parts' ETags -- to
    tests/s3_mock_server.py, which re-hashes every body (hashlib), verifies every SigV4
    signature and answers the object's multipart ETag; every pass's object ETag must equal the
    one hashlib's part MD5s give.  Wall-clock of the whole pass (create + hash + upload +
    complete; --repeat: the last pass) for the
    GPU batch (one call, and one call per job: merged on the device), the CPU SHA-NI drop-in
    and its scalar loop (lib/hash-like cost), the size-aware route (--route auto: the measured
    model picks the GPU, the CPU drop-in or the split for the batch; `auto_route` says which),
    the same three with Content-MD5 as well (`*_md5`: both digests per part; AUTO priced for
    both, `auto_md5_route`), plus the GPU hash alone."""
    import re
    import subprocess
    import tempfile
    import urllib.request
    app = os.path.join(ROOT, "apps", "build", "s3-upload-hash")
    end = int(offs[nparts - 1] + lens[nparts - 1])
    if not os.path.exists(app) or int(offs[nparts - 1]) != (nparts - 1) * int(lens[0]):
        return {"error": "app not built or parts not contiguous"}
    res = {"workload": f"{nparts} x 8 MiB (C2 parts 0-{nparts - 1}) in one file, {jobs} jobs x "
                       f"{nparts // jobs} parts; CreateMultipartUpload, hash + signed UploadPart "
                       "PUT per part, CompleteMultipartUpload, to a loopback mock S3 endpoint "
                       "that re-hashes bodies, verifies SigV4 and answers the object ETag",
           "repeat": repeat, "seconds": {}}
    srv = None
    with tempfile.TemporaryDirectory(dir="/tmp") as td:
        path = os.path.join(td, "object.bin")
        data[:end].cpu().numpy().tofile(path)
        try:
            srv = subprocess.Popen([sys.executable, os.path.join(ROOT, "tests", "s3_mock_server.py"),
                                    "--port", "0"], stdout=subprocess.PIPE,
                                   stderr=subprocess.DEVNULL, text=True)
            url = f"http://127.0.0.1:{int(srv.stdout.readline())}"
            want = [s3_hex(gd[k]) for k in range(nparts)]
            # the object ETag S3 computes: MD5 of the parts' binary MD5s + "-" + count (hashlib)
            import hashlib
            from concurrent.futures import ThreadPoolExecutor
            host = np.fromfile(path, dtype=np.uint8)
            pb = int(lens[0])
            with ThreadPoolExecutor(16) as ex:
                md5s = list(ex.map(lambda k: hashlib.md5(host[k * pb:(k + 1) * pb]).digest(),
                                   range(nparts)))
            del host
            res["object_etag_expected"] = f"{hashlib.md5(b''.join(md5s)).hexdigest()}-{nparts}"
            etags = {}
            send = ["--send", "--multipart"]
            for name, extra, env in (("gpu", send, {}),
                                     ("gpu_per_job", send + ["--per-job"], {}),
                                     ("cpu_shani", send + ["--cpu"], {}),
                                     ("cpu_scalar", send + ["--cpu"], {"S3H_CPU_SCALAR": "1"}),
                                     ("auto", send + ["--route", "auto"], {}),
                                     # both upload headers (Content-MD5 + x-amz-content-sha256):
                                     # AUTO prices the CPU side with MD5 too (round 6)
                                     ("gpu_md5", send + ["--content-md5"], {}),
                                     ("cpu_shani_md5", send + ["--cpu", "--content-md5"], {}),
                                     ("auto_md5", send + ["--route", "auto", "--content-md5"], {}),
                                     ("gpu_hash_only", [], {})):
                r = subprocess.run([app, "-f", path, "-j", str(jobs), "-n", str(nparts // jobs),
                                    "--endpoint", url, "--repeat", str(repeat), *extra],
                                   capture_output=True, text=True, timeout=300,
                                   env={**os.environ, **env})
                m = re.search(r"in ([\d.]+) s = ", r.stderr)
                got = [l.split(",")[4] for l in r.stdout.strip().splitlines()[1:]]
                if r.returncode != 0 or not m or got != want:
                    res["error"] = f"{name}: rc {r.returncode}, digests match {got == want}"
                    break
                res["seconds"][name] = float(m.group(1))
                if extra:
                    me = re.search(r"object etag (\S+)", r.stderr)
                    etags[name] = me.group(1) if me else None
                if name in ("auto", "auto_md5"):
                    ra = re.search(r"route auto -> (\w+)", r.stderr)
                    res[f"{name}_route"] = ra.group(1) if ra else None
            with urllib.request.urlopen(url + "/stats", timeout=10) as f:
                res["server"] = json.loads(f.read())
            res["object_etags_match"] = bool(etags) and all(
                e == res["object_etag_expected"] for e in etags.values())
            if "error" not in res and not res["object_etags_match"]:
                res["error"] = f"object ETags {etags} != {res['object_etag_expected']}"
        except (OSError, ValueError, subprocess.SubprocessError) as e:
            res["error"] = repr(e)
        finally:
            if srv is not None:
                srv.kill()
                srv.wait()
    res["digests_match_device_run"] = "error" not in res
    return res


def s3_hex(words) -> str:
    return np.ascontiguousarray(words, dtype=np.uint32).tobytes().hex()


def c4_shard(args, s3, torch, dist, dev, rank, world, local, ident, ph, steps: int = 3):
    """BASELINE config 4 beside the C2 headline of a multi-GPU run: 8,192 x 8 MiB per GPU,
    global part p on rank p % N (65,536 parts = 512 GiB at N = 8), no collective on the data
    path.  The AUTO kernel (skews: producers on their consumers' SIMDs, ~1.4 kW per board) and
    skewp (~0.7 kW) are timed on the same parts, each with the clock probe and the board power
    (amdsmi) per GPU, so the node's power envelope decides between them on measured numbers;
    per-GPU and aggregate GiB/s over the max-over-ranks time, fixture parity on every rank
    (four own-shard fixtures per rank).  A device fault on any rank raises DeviceFault on
    every rank together (status_all)."""
    from s3client_amd.shard import shard_ids
    per, L = 8192, 8 * MIB
    ids = shard_ids(per * world, rank, world)
    lens = np.full(per, L, dtype=np.uint64)
    offs = np.arange(per, dtype=np.uint64) * np.uint64(L)
    data = torch.empty(per * L, dtype=torch.uint8, device=dev)
    s3.generate_parts(data, offs, lens, ids, SEED)
    stream = torch.cuda.current_stream(dev)
    fx = golden_fixtures("c4", "sha256")
    gib_gpu = per * L * steps / 2**30
    algo = per * (L + 32)  # bytes read once + digests written, per GPU per launch
    with s3.Plan(offs, lens, device=local) as p:  # AUTO under the current (default) policy
        auto_kernel = p.info()["kernel"]
    res = {"workload": f"C4: {per} x 8 MiB per GPU, {per * world} parts over {world} GPUs "
                       "(part p on rank p % N)", "steps": steps, "kernels": {}, "kernel": auto_kernel}
    ph.mark("c4 generate")
    for kern in ("skews", "skewp"):  # both C4 kernels whatever AUTO's policy picks
        plan = s3.Plan(offs, lens, device=local, kernel=kern)
        info = plan.info()
        out = torch.zeros((per, 8), dtype=torch.int32, device=dev)
        plan.launch(data, out, stream)
        status_all(dist, world, lambda: plan.status(stream))
        dist.barrier()
        torch.cuda.synchronize(dev)
        with power_sampler(ident) as pw:
            t0 = time.perf_counter()
            for _ in range(steps):
                plan.launch(data, out, stream)
            torch.cuda.synchronize(dev)
            mine = time.perf_counter() - t0
            dist.barrier()
            wall = time.perf_counter() - t0
        status_all(dist, world, lambda: plan.status(stream))
        probe = clock_probe(torch, plan, info, data, out, stream, dev) or {}
        gd = out.cpu().numpy().view(np.uint32)
        chk = [k for k, p in enumerate(ids) if int(p) in fx]
        bad = sum(s3.hash_to_text(gd[k]) != fx[int(ids[k])] for k in chk)
        plan.close()
        pws = gather_obj(dist, world, pw.summary())
        # per rank: time (us), wall (us), fixtures checked, mismatches, clock (MHz), cycles/block
        r = per_rank(dist, world, [int(mine * 1e6), int(wall * 1e6), len(chk), int(bad),
                                   int(probe.get("clock_GHz", 0) * 1e3),
                                   int(probe.get("cycles_per_block", 0))])
        t_rank = [x[0] / 1e6 for x in r]
        res["kernels"][info["kernel"]] = {
            "per_gpu_GiBps": [round(gib_gpu / t, 3) for t in t_rank],
            "aggregate_GiBps": round(gib_gpu * world / max(max(t_rank), max(x[1] for x in r) / 1e6), 3),
            "ms_per_step_max_rank": round(1e3 * max(t_rank) / steps, 3),
            "hbm_roofline_frac_per_gpu": [round(algo * steps / t / 1e9 / HBM_PEAK_GBS, 5)
                                          for t in t_rank],
            "clock_GHz_per_gpu": [x[4] / 1e3 for x in r],
            "cycles_per_block_per_gpu": [x[5] for x in r],
            "board_W_busy_mean_per_gpu": [p.get("busy_mean_W") for p in pws],
            "J_per_GiB_per_gpu": [energy(p, gib_gpu / t).get("J_per_GiB")
                                  for p, t in zip(pws, t_rank)],
            "board_W_max_per_gpu": [p.get("max_W") for p in pws],
            "parity": {"fixtures_checked": sum(x[2] for x in r), "mismatches": sum(x[3] for x in r),
                       "fixtures_checked_per_rank": [x[2] for x in r]}}
        ph.mark(f"c4 {info['kernel']}")
    del data
    torch.cuda.empty_cache()
    auto = res["kernels"][res["kernel"]]
    res.update({k: auto[k] for k in ("per_gpu_GiBps", "aggregate_GiBps", "ms_per_step_max_rank",
                                     "hbm_roofline_frac_per_gpu", "parity")})
    res["faster_kernel"] = max(res["kernels"], key=lambda k: res["kernels"][k]["aggregate_GiBps"])
    res["board_power_cap_W"] = s3.device_power_cap(local)
    return res


def shared_buffer_views(h, per: int, ndev: int, L: int) -> list:
    """host_resident_multi's parts: global part i = buffer part i // ndev, so the host path's
    split (part i on device i % ndev) gives every device buffer parts 0..per-1 in order, at the
    buffer's constant stride L (its 2-D copy form).  `h` is one buffer, or a list of ndev
    buffers (device d reads h[d]: the buffer on its own NUMA node)."""
    pick = (lambda i: h[i % ndev]) if isinstance(h, list) else (lambda i: h)
    return [pick(i)[(i // ndev) * L:(i // ndev + 1) * L] for i in range(per * ndev)]


def host_resident_multi(s3, torch, dev, world: int, ph, per: int = 1024, reps: int = 3):
    """Rank 0 of an N-GPU run: the C2 weak-scaling job (1,024 x 8 MiB per GPU) starting and
    ending in HOST memory, through s3h_sha256_batch_host(..., ndevices=N) -- part i on device
    i % N, one host thread per device -- with every H2D copy inside the timed region.

    Bounded host memory: ONE pinned buffer of 1,024 parts (8 GiB, C2 ids 0..1023) per NUMA
    node in use, allocated on that node (s3h_host_alloc), whatever N; global part i is part
    i // N of the buffer on device i % N's node, so every device hashes all 1,024 buffer parts
    (the same per-device work as the device-resident line) from its own socket's memory, as an
    uploader staging each device's parts on its node would.  Parity: every device's digest of
    buffer part j equals every other's, and the C2 fixtures pin parts 0..15, 511, 1022, 1023."""
    L = 8 * MIB
    ndev = min(world, torch.cuda.device_count())
    n = per * ndev
    t_setup = time.perf_counter()
    dev_nodes = [s3.device_numa(d)["node"] for d in range(ndev)]
    bufs = {}
    buf = torch.empty(per * L, dtype=torch.uint8, device=dev)
    lens = np.full(per, L, dtype=np.uint64)
    offs = np.arange(per, dtype=np.uint64) * np.uint64(L)
    s3.generate_parts(buf, offs, lens, np.arange(per), SEED)
    try:
        for node in sorted(set(dev_nodes)):
            pb, t = pinned_on(s3, torch, per * L, node)
            t.copy_(buf)
            bufs[node] = (pb, t)
    except Exception as e:  # noqa: BLE001 -- reported in the line
        return {"error": f"pinned host buffer of {per * L / 2**30:.0f} GiB per node: {e}"}
    del buf
    torch.cuda.empty_cache()
    views = shared_buffer_views([bufs[dev_nodes[d]][0].array for d in range(ndev)], per, ndev, L)
    buffer_nodes = {str(k): s3.mem_node(v[1]) for k, v in bufs.items()}
    setup = time.perf_counter() - t_setup
    ph.mark(f"host_resident setup ({len(bufs)} x 8 GiB pinned, one per NUMA node)")
    out = s3.sha256_batch_host(views, ndevices=ndev)  # warm: a cached context per device
    times = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = s3.sha256_batch_host(views, ndevices=ndev)
        times.append(time.perf_counter() - t0)
    fx = golden_fixtures("c2", "sha256")
    chk = [j for j in range(per) if j in fx]
    bad = sum(s3.hash_to_text(out[j * ndev]) != fx[j] for j in chk)
    same = bool((out.reshape(per, ndev, 8) == out.reshape(per, ndev, 8)[:, :1]).all())
    threads, cpus = s3.host_threads(ndev)
    gib = n * L / 2**30
    shard_cpus = [s3.host_numa_info(d)["bound_cpus"] for d in range(ndev)]
    del bufs, views
    s3.trim()
    return {"metric": f"host-resident (H2D-inclusive) SHA-256 GiB/s over {ndev} GPU(s)",
            "value": round(gib / float(np.mean(times)), 3), "best": round(gib / min(times), 3),
            "per_gpu": round(gib / float(np.mean(times)) / ndev, 3), "unit": "GiB/s",
            "devices": ndev, "parts": n, "parts_per_device": per, "reps": reps,
            "pinned_host_GiB": per * L / 2**30 * len(buffer_nodes),
            "numa": {"device_nodes": dev_nodes, "buffer_nodes": buffer_nodes,
                     "shard_thread_cpus_per_device": shard_cpus,
                     "layout": "one 8 GiB pinned buffer per NUMA node in use; each device reads "
                               "the buffer on its own node, its shard thread bound to that "
                               "node's CPUs"},
            "ms_per_batch": round(1e3 * float(np.mean(times)), 2), "setup_s": round(setup, 2),
            "path": "pinned host parts -> per-device 3-slot HBM ring (one 2-D H2D copy per "
                    "256 KiB slice) -> skew kernel per slice -> digests D2H "
                    "(s3h_sha256_batch_host, one host thread per device, on its node)",
            "host_cpus": cpus, "staging_threads_per_device": threads,
            "fixtures_checked": len(chk), "fixture_mismatches": int(bad),
            "digests_match_across_devices": same}


def host_mode(args, s3, torch, dist, data, ids, lens, offs, world, rank, name):
    """H2D-inclusive rate: parts start in pinned host memory, digests end in host memory."""
    end = int(offs[-1] + lens[-1])
    host = torch.empty(end, dtype=torch.uint8, pin_memory=True)
    host.copy_(data[:end])
    del data
    torch.cuda.empty_cache()
    h = host.numpy()
    views = [h[int(o):int(o) + int(L)] for o, L in zip(offs, lens)]
    dual = args.mode == "host-dual"

    def run():
        if dual:
            return s3.sha256_md5_batch_host(views, ndevices=1, slice_bytes=args.slice_bytes)
        return s3.sha256_batch_host(views, ndevices=1, slice_bytes=args.slice_bytes), None

    out, m5 = run()
    times = []
    for _ in range(max(1, args.steps)):
        t0 = time.perf_counter()
        out, m5 = run()
        times.append(time.perf_counter() - t0)
    wall = float(np.mean(times))
    bad = _fixture_mismatches(s3, ids, out, m5, args.config, args.part_bytes)
    if rank == 0:
        what = "SHA-256 + MD5 (one H2D pass)" if dual else "SHA-256"
        print(json.dumps({"metric": f"host-resident (H2D-inclusive) {what} GiB/s", "value":
                          round(float(lens.sum()) / 2**30 / wall, 3), "unit": "GiB/s",
                          "n_gpus": 1, "steps": args.steps,
                          "config": {"workload": name, "slice_bytes": args.slice_bytes or "auto"},
                          "fixture_mismatches": int(bad), "ms_per_batch": round(wall * 1e3, 2)}))
    return 0


def golden_fixtures(cfg: str, algo: str, part_bytes: int = 0) -> dict:
    """{global part id: hex digest} of the committed lib/hash fixtures that apply to this
    workload's parts: generator-G 8 MiB parts (C2 / C4 ids and four parts of every rank's
    shard at N = 2, 4, 8; MD5: the C2 ids) or the C3 parts; none for a --part-bytes
    override."""
    if part_bytes:
        return {}
    with open(os.path.join(ROOT, "tests", "golden", "sha256_golden.json")) as f:
        gold = json.load(f)
    if algo == "md5":
        src = gold["md5"]["c3_parts"] if cfg == "c3" else gold["md5"]["c2_parts"]
    else:
        src = (gold["c3_parts"] if cfg == "c3"
               else gold["c2_parts"] + gold["c4_parts"] + gold["shard_parts"])
    return {e["p"]: e["digest"] for e in src}


def _fixture_mismatches(s3, ids, sha, m5=None, cfg: str = "c2", part_bytes: int = 0) -> int:
    """Digests of the workload's parts that have committed golden fixtures, compared with them."""
    fixtures = golden_fixtures(cfg, "sha256", part_bytes)
    bad = sum(s3.hash_to_text(sha[s]) != fixtures[int(p)] for s, p in enumerate(ids)
              if int(p) in fixtures)
    if m5 is not None:
        mf = golden_fixtures(cfg, "md5", part_bytes)
        bad += sum(s3.digests_to_text(m5[s:s + 1], 4)[0] != mf[int(p)] for s, p in enumerate(ids)
                   if int(p) in mf)
    return int(bad)


def dual_mode(args, s3, torch, data, ids, lens, offs, rank, name, stream):
    """Device-resident SHA-256 + MD5 of every part (s3h_sha256_md5_batch_device: the MD5
    kernel on a side stream beside the SHA-256 one), wall time per batch incl. the join."""
    sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
    torch.cuda.synchronize()
    times = []
    for _ in range(max(1, args.steps)):
        t0 = time.perf_counter()
        sha, m5 = s3.sha256_md5_batch_device(data, offs, lens, stream=stream)
        times.append(time.perf_counter() - t0)
    wall = float(np.mean(times))
    bad = _fixture_mismatches(s3, ids, sha.cpu().numpy().view(np.uint32),
                              m5.cpu().numpy().view(np.uint32), args.config, args.part_bytes)
    if rank == 0:
        print(json.dumps({"metric": "device-resident SHA-256 + MD5 GiB/s (both digests)",
                          "value": round(float(lens.sum()) / 2**30 / wall, 3), "unit": "GiB/s",
                          "n_gpus": 1, "steps": args.steps, "config": {"workload": name},
                          "fixture_mismatches": bad, "ms_per_batch": round(wall * 1e3, 2)}))
    return 0


def stream_mode(args, s3, torch, data, ids, lens, offs, rank, name, stream):
    """Each part as one streamed object: appended in --chunk-bytes chunks (any size, so the
    carried partial blocks are exercised when it is not a multiple of 64), then finished."""
    n = len(lens)
    algo = args.algo
    st = s3.Stream(n, device=torch.cuda.current_device(), algo=algo, kernel=args.kernel)
    out = torch.zeros((n, st.words), dtype=torch.int32, device=data.device)
    cb = args.chunk_bytes
    nupd = int((int(lens.max()) + cb - 1) // cb)
    src = args.stream_source
    host = None
    if src != "device":  # the parts in host memory: each update copies its chunks (H2D included)
        end = int(offs[-1] + lens[-1])
        host = torch.empty(end, dtype=torch.uint8, pin_memory=(src == "pinned"))
        host.copy_(data[:end])
        host_out = np.zeros((n, st.words), dtype=np.uint32)

    def one_object_pass():
        for k in range(nupd):
            lk = np.minimum(np.maximum(lens.astype(np.int64) - k * cb, 0), cb).astype(np.uint64)
            if host is None:
                st.update_device(data, offs + np.uint64(k * cb), lk, stream)
            else:
                st.update(s3.BufferParts(host, offs + np.uint64(k * cb), lk))
        if host is None:
            st.final_device(out, stream)
        else:
            host_out[:] = st.final()
            out.copy_(torch.from_numpy(host_out.view(np.int32)))

    for _ in range(args.warmup):
        one_object_pass()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_object_pass()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / max(1, args.steps)
    st.status(stream)  # every update/final launch's device error word clear (raises otherwise)
    gd = out.cpu().numpy().view(np.uint32)
    fixtures = golden_fixtures(args.config, algo, args.part_bytes)
    checked = [int(p) for p in ids if int(p) in fixtures]
    bad = sum(s3.hash_to_text(gd[s]) != fixtures[int(p)]
              for s, p in enumerate(ids) if int(p) in fixtures)
    if rank == 0:
        print(json.dumps({"metric": f"streamed-object {algo.upper()} GiB/s (s3h_stream_*, "
                          "device-resident chunks; SURVEY 8(f).2, not the metric)",
                          "value": round(float(lens.sum()) / 2**30 / wall, 3), "unit": "GiB/s",
                          "n_gpus": 1, "steps": args.steps,
                          "config": {"workload": name, "objects": n, "chunk_bytes": cb,
                                     "updates_per_object": nupd, "chunks_from": src},
                          "parity": {"fixtures_checked": len(checked), "mismatches": int(bad)},
                          "ms_per_pass": round(wall * 1e3, 2)}))
    st.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
