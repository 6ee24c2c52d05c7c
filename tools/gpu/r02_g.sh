#!/bin/bash
# Round-2 GPU pass G: which half of sha256_md5_group_kernel is slow on C4 (8,192 x 8 MiB)?
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "dual" --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu_g.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_g.log; [ $rc -eq 0 ] || exit 1
for v in default grp_sha grp_md5 md5d2 md5d12; do
  lib=tools/exp/libs3hash_$v.so; [ $v = default ] && lib=s3client_amd/lib/libs3hash.so
  S3H_LIBRARY=$lib timeout -k 10 200 python bench.py --mode dual --config c4 --steps 3 > gpurun_out/g_$v.jsonl 2> gpurun_out/g_$v.err || exit 1
  echo "$v $(cut -c1-200 gpurun_out/g_$v.jsonl | grep -o '"value": [0-9.]*\|"ms_per_batch": [0-9.]*\|"fixture_mismatches": [0-9]*' | tr '\n' ' ')"
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_dual_c4 -o run --output-format csv -- python3 bench.py --mode dual --config c4 --steps 2 > /dev/null 2>&1 || exit 1
head -4 gpurun_out/prof_dual_c4/run_kernel_stats.csv | cut -c1-160
