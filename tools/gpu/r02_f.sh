#!/bin/bash
# Round-2 GPU pass F: self-fed MD5 wave in the SHA-256 + MD5 group kernel (skewp range).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_f.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_f.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_f.log | head -20; exit 1; }
for cfg in c4 c2; do
  timeout -k 10 200 python bench.py --mode dual --config $cfg --steps 3 > gpurun_out/f_dual_$cfg.jsonl 2> gpurun_out/f_dual_$cfg.err || exit 1
  cat gpurun_out/f_dual_$cfg.jsonl
done
timeout -k 10 200 python bench.py --mode host-dual --config c2 --steps 3 > gpurun_out/f_hostdual_c2.jsonl 2> gpurun_out/f_hostdual_c2.err || exit 1
cat gpurun_out/f_hostdual_c2.jsonl
