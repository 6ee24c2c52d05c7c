#!/bin/bash
# Quad-kernel consumer-waves sweep (S3H_QUAD_WAVES) vs the pair kernel, plus C3/C4.
set -e
out=gpurun_out/sweep_quad_waves3.jsonl
mkdir -p gpurun_out && rm -f $out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_sweep.log 2>&1 || { tail -20 gpurun_out/pytest_sweep.log; exit 1; }
tail -1 gpurun_out/pytest_sweep.log
for w in 1 2 3 4; do
  for n in 2048 4096 8192; do
    S3H_QUAD_WAVES=$w timeout -k 10 120 python bench.py --kernel quad --parts-per-gpu $n --part-bytes 262144 \
      --steps 5 --warmup 2 --no-cpu-baseline | sed "s/^{/{\"quad_waves\": $w, /" >> $out
  done
done
for n in 2048 4096 8192 16384; do
  timeout -k 10 120 python bench.py --kernel pair --parts-per-gpu $n --part-bytes 262144 --steps 5 --warmup 2 \
    --no-cpu-baseline >> $out
done
for w in 2 4; do
  S3H_QUAD_WAVES=$w timeout -k 10 300 python bench.py --config c4 --kernel quad --steps 3 --warmup 1 --no-cpu-baseline \
    | sed "s/^{/{\"quad_waves\": $w, /" >> $out
done
timeout -k 10 300 python bench.py --config c4 --kernel pair --steps 3 --warmup 1 --no-cpu-baseline >> $out
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline >> $out
python3 - <<'PY'
import json
for l in open("gpurun_out/sweep_quad_waves3.jsonl"):
    d = json.loads(l)
    print(d.get("quad_waves", "-"), d["config"]["kernel"], d["config"]["parts_per_gpu"], d["config"]["part_bytes"], d["value"], d["issue"]["cycles_per_block"])
PY
