#!/bin/bash
# Round-2 GPU pass AG: the denormal-multiply producer as the product (tools/gen_producer.py):
# full GPU suite, C4 shard skews x2 + skewp on the same box, amd-smi power during one skews run.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_ag.txt 2>&1 || { tail -40 gpurun_out/pytest_gpu_ag.txt; exit 1; }
tail -3 gpurun_out/pytest_gpu_ag.txt
bench() {  # tag kernel
  timeout -k 10 300 python bench.py --config c4 --kernel $2 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ag_$1.jsonl 2> gpurun_out/bench_ag_$1.err || { tail -5 gpurun_out/bench_ag_$1.err; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ag_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['value'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
}
bench skews1 skews
( for i in $(seq 1 300); do amd-smi metric -g 0 -p -c -t 2>/dev/null | tr -s ' \n' ' '; echo; sleep 0.1; done ) > gpurun_out/smi_ag_skews.txt 2>&1 &
MON=$!
bench skews2 skews; rc=$?
kill $MON 2>/dev/null; wait $MON 2>/dev/null
[ $rc -eq 0 ] || exit 1
bench skewp skewp
