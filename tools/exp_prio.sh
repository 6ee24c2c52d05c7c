#!/bin/bash
# Experiment: pacer microbenchmark + quad-kernel wave-priority schemes at NC = 1..4.
set -e
mkdir -p gpurun_out
timeout -k 10 150 ./tools/ubench_cu_waves > gpurun_out/cu_waves2.txt 2>&1
grep pacer gpurun_out/cu_waves2.txt
out=gpurun_out/exp_prio.jsonl; rm -f $out
for p in 0 1 2; do
  for w in 1 2 3; do
    S3H_PRIO=$p S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --parts-per-gpu 2048 \
      --part-bytes 262144 --steps 5 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"prio\": $p, \"nc\": $w, /" >> $out
  done
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print('prio', d['prio'], 'nc', d['nc'], d['value'], d['issue']['cycles_per_block'])
"
