#!/bin/bash
# Quad-kernel consumer-waves sweep (S3H_QUAD_WAVES) vs the pair kernel; run on the GPU box.
set -e
out=gpurun_out/sweep_quad_waves2.jsonl
mkdir -p gpurun_out && rm -f $out
for w in 1 2 3 4; do
  for n in 2048 4096 8192 16384; do
    S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --parts-per-gpu $n --part-bytes 262144 \
      --steps 5 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"quad_waves\": $w, /" >> $out
  done
done
for w in 2 4; do
  S3H_QUAD_WAVES=$w timeout -k 10 300 python bench.py --config c4 --kernel quad --steps 3 --warmup 1 --no-cpu-baseline \
    | sed "s/^{/{\"quad_waves\": $w, /" >> $out
done
timeout -k 10 300 python bench.py --config c4 --kernel pair --steps 3 --warmup 1 --no-cpu-baseline >> $out
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline >> $out
python3 - <<'PY'
import json
for l in open("gpurun_out/sweep_quad_waves2.jsonl"):
    d = json.loads(l)
    print(d.get("quad_waves", "-"), d["config"]["kernel"], d["config"]["parts_per_gpu"], d["config"]["part_bytes"], d["value"])
PY
