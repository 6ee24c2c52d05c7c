#!/bin/bash
# Round-2 GPU pass T: full regression on the current tree -- GPU suite, smoke, default bench
# line (C2), C3 (solo workgroups, rocprofv3 stats) and C4 (shared-SIMD kernel vs skewp).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_t.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_t.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_t.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_t.log 2>&1 || { tail -20 gpurun_out/smoke_t.log; exit 1; }
tail -1 gpurun_out/smoke_t.log
timeout -k 10 300 python bench.py > gpurun_out/bench_t.jsonl 2> gpurun_out/bench_t.err || { tail -20 gpurun_out/bench_t.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_t.jsonl').read().strip().splitlines()[-1]); print('C2', d['value'], d['roofline']['frac'], d['issue']['frac'], d['host_resident']['value'], d['cpu_baseline']['value'], d['parity'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3_t -o run --output-format csv -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_t.jsonl 2> gpurun_out/bench_c3_t.err || { tail -5 gpurun_out/bench_c3_t.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_c3_t.jsonl').read().strip().splitlines()[-1]); print('C3', d['value'], d['config']['solo_workgroups'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['frac'], d['parity'])"
head -2 gpurun_out/prof_c3_t/run_kernel_stats.csv | cut -c1-140
for k in auto skewp; do
  timeout -k 10 300 python bench.py --config c4 --kernel $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_t_$k.jsonl 2> gpurun_out/bench_c4_t_$k.err || { tail -20 gpurun_out/bench_c4_t_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_c4_t_$k.jsonl').read().strip().splitlines()[-1]); print('C4', d['config']['kernel'], d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
done
