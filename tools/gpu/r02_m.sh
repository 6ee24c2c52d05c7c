#!/bin/bash
# Round-2 GPU pass M: solo workgroups for the two-group skew kernel -- full GPU suite (incl.
# the new solo-grid test and full C3), smoke, C3 bench line and its rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_m.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_m.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_m.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_m.log 2>&1 || { tail -20 gpurun_out/smoke_m.log; exit 1; }
tail -1 gpurun_out/smoke_m.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_solo -o run --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_solo.jsonl 2> gpurun_out/bench_c3_solo.err || { tail -20 gpurun_out/bench_c3_solo.err; exit 1; }
tail -c 600 gpurun_out/bench_c3_solo.jsonl
head -3 gpurun_out/prof_c3_solo/run_kernel_stats.csv | cut -c1-200
