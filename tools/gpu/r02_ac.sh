#!/bin/bash
# Round-2 GPU pass AC: skew-layout group kernel (SHA-256 skew group + self-fed MD5 wave of the
# same 8 parts, experiment build) vs the product's split grid / skewp group kernel, <= 2,048 parts.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S3H_LIBRARY=tools/exp/libs3hash_groupskew.so timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "dual" --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_ac.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_ac.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_ac.log | head -20; exit 1; }
S3H_LIBRARY=tools/exp/libs3hash_groupskew.so timeout -k 10 400 python tools/sweep_parts.py --counts 64,1024,1500,1821,2047 > gpurun_out/sweep_ac_groupskew.jsonl 2> gpurun_out/sweep_ac.err || { tail -5 gpurun_out/sweep_ac.err; exit 1; }
cat gpurun_out/sweep_ac_groupskew.jsonl
