#!/bin/bash
# Experiment: shadow consumers (identical instruction stream in lockstep) for the quad kernel.
set -e
mkdir -p gpurun_out
out=gpurun_out/exp_shadow.jsonl; rm -f $out
for sh in 0 1; do
  S3H_QUAD_SHADOW=$sh timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu-baseline \
    | sed "s/^{/{\"shadow\": $sh, /" >> $out
  for w in 1 2; do
    S3H_QUAD_SHADOW=$sh S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --parts-per-gpu 2048 \
      --part-bytes 262144 --steps 5 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"shadow\": $sh, \"nc\": $w, /" >> $out
  done
done
python3 -c "
import json
for l in open('$out'):
    d = json.loads(l); print('shadow', d['shadow'], 'nc', d.get('nc', 'auto'), d['config']['parts_per_gpu'], d['value'], d['issue']['cycles_per_block'], d['parity'])
"
