#!/bin/bash
# Round-2 GPU pass I (final kernels; same as pass B): rocprofv3 kernel stats + HBM / SQ PMC passes for the shipped AUTO
# kernels on C2 (skew), C4 rank-0 shard (skewp) and C3 (skew NC=2); co-issue priority
# variants; the upload app's CPU drop-in with 16 job threads (the host's CPU share).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --no-host-resident"
prof() {  # name, steps, bench args...
  local name=$1 steps=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python3 bench.py --steps $steps --warmup 1 $B "$@" > gpurun_out/prof_$name.jsonl 2> gpurun_out/prof_$name.err || return 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${name}_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${name}_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_${name}_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  echo "prof $name done"; tail -c 400 gpurun_out/prof_$name.jsonl
}
prof c2 5 --config c2 || exit 1
prof c4 3 --config c4 || exit 1
prof c3 2 --config c3 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dual_c4 -o run --output-format csv -- python3 bench.py --mode dual --config c4 --steps 3 > gpurun_out/prof_dual_c4.jsonl 2>/dev/null || exit 1
head -3 gpurun_out/prof_dual_c4/run_kernel_stats.csv | cut -c1-150
