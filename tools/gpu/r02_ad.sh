#!/bin/bash
# Round-2 GPU pass AD: dual-digest routing (split / skew group / skewp group) -- dual tests and
# the part-count sweep on the product.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "dual" --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_ad.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_ad.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_ad.log | head -20; exit 1; }
timeout -k 10 600 python tools/sweep_parts.py --counts 1024,1800,1821,2047,2049,4097,8192 > gpurun_out/sweep_ad.jsonl 2> gpurun_out/sweep_ad.err || { tail -5 gpurun_out/sweep_ad.err; exit 1; }
cat gpurun_out/sweep_ad.jsonl
