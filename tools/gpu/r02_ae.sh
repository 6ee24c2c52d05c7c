#!/bin/bash
# Round-2 GPU pass AE: power / clock telemetry (amd-smi, sampled ~10/s) while the C4 shard runs
# on the shared-SIMD kernel and on skewp -- is the skews clock drop a power limit?
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
( which amd-smi && amd-smi metric --help | head -30 ) > gpurun_out/smi_help.txt 2>&1 || true
for k in skews skewp; do
  ( for i in $(seq 1 400); do amd-smi metric -g 0 -p -c -t 2>/dev/null | tr -s ' \n' ' '; echo; sleep 0.1; done ) > gpurun_out/smi_$k.txt 2>&1 &
  MON=$!
  timeout -k 10 300 python bench.py --config c4 --kernel $k --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/bench_ae_$k.jsonl 2> gpurun_out/bench_ae_$k.err; rc=$?
  kill $MON 2>/dev/null; wait $MON 2>/dev/null
  [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_ae_$k.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_ae_$k.jsonl').read().strip().splitlines()[-1]); print('$k', d['value'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'])"
done
head -c 1500 gpurun_out/smi_skews.txt
