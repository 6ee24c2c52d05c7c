#!/bin/bash
# Quad-kernel consumer-waves sweep (S3H_QUAD_WAVES) vs the pair kernel; run on the GPU box.
set -e
out=gpurun_out/sweep_quad_waves.jsonl
mkdir -p gpurun_out && rm -f $out
for w in 1 2 3 4; do
  S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --steps 5 --warmup 2 --no-cpu-baseline \
    | sed "s/^{/{\"quad_waves\": $w, /" >> $out
  for n in 2048 4096 8192 16384; do
    S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --parts-per-gpu $n --part-bytes 262144 \
      --steps 5 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"quad_waves\": $w, /" >> $out
  done
done
for n in 2048 4096 8192 16384; do
  timeout -k 10 120 python bench.py --kernel pair --parts-per-gpu $n --part-bytes 262144 --steps 5 --warmup 2 \
    --no-cpu-baseline >> $out
done
python3 - <<'PY'
import json
for l in open("gpurun_out/sweep_quad_waves.jsonl"):
    d = json.loads(l)
    print(d.get("quad_waves", "-"), d["config"]["kernel"], d["config"]["parts_per_gpu"], d["config"]["part_bytes"], d["value"])
PY
