#!/bin/bash
# Round-2 GPU pass V: stream plans re-planning solo workgroups per update (plan_refill).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_configs.py -m gpu -x -v -k "stream or solo" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_v.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_v.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_v.log | head -20; exit 1; }
