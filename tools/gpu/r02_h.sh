#!/bin/bash
# Round-2 GPU pass H: self-fed MD5 with a branch-free fast loop in the SHA-256 + MD5 group kernel.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_programs.py -m gpu -x -q -k "dual or md5 or sha256_md5" --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_h.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_h.log; [ $rc -eq 0 ] || exit 1
for cfg in c4 c2; do
  timeout -k 10 200 python bench.py --mode dual --config $cfg --steps 3 > gpurun_out/h_dual_$cfg.jsonl 2> gpurun_out/h_dual_$cfg.err || exit 1
  echo "$cfg $(grep -o '"value": [0-9.]*\|"ms_per_batch": [0-9.]*\|"fixture_mismatches": [0-9]*' gpurun_out/h_dual_$cfg.jsonl | tr '\n' ' ')"
done
