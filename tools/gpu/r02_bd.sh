#!/bin/bash
# Round-2 GPU pass BD: regression at HEAD (dual file parts, Content-MD5, download verify) -- full GPU suite,
# smoke, default bench line, rocprofv3 kernel stats of the default bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_bd.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_bd.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_bd.log | head -20; exit 1; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_bd.log 2>&1 || { tail -20 gpurun_out/smoke_bd.log; exit 1; }
tail -1 gpurun_out/smoke_bd.log
timeout -k 10 300 python bench.py > gpurun_out/bench_bd.jsonl 2> gpurun_out/bench_bd.err || { tail -20 gpurun_out/bench_bd.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_bd.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['issue']['frac'], d['host_resident']['value'], d['cpu_baseline']['value'], d['parity'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2_bd -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-host-resident > gpurun_out/prof_c2_bd.jsonl 2> gpurun_out/prof_c2_bd.err || { tail -5 gpurun_out/prof_c2_bd.err; exit 1; }
head -3 gpurun_out/prof_c2_bd/run_kernel_stats.csv | cut -c1-160
