#!/bin/bash
# Round-2 GPU pass AI: C3 solo workgroups on the barrier body (S3H_EXP_SOLO_BARRIER, experiment
# build) vs the product's flag-synchronised body, alternating on one box.
# (The experiment, removed after this measurement: in sha256_skew_pairs_kernel, for b < A.solo,
# skew_body<1, false, false>(A, b, wave >> 1, L[0], nullptr) instead of the flag body.)
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S3H_LIBRARY=tools/exp/libs3hash_solobar.so timeout -k 10 200 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_configs.py -k "solo or c3" > gpurun_out/ai_pytest.txt 2>&1 || { tail -30 gpurun_out/ai_pytest.txt; exit 1; }
tail -1 gpurun_out/ai_pytest.txt
for i in 1 2; do
  for v in prod solobar; do
    if [ $v = prod ]; then L=s3client_amd/lib/libs3hash.so; else L=tools/exp/libs3hash_$v.so; fi
    S3H_LIBRARY=$L timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-resident > gpurun_out/bench_ai_${v}_$i.jsonl 2> gpurun_out/bench_ai_${v}_$i.err || { tail -5 gpurun_out/bench_ai_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_ai_${v}_$i.jsonl').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
  done
done
