#!/bin/bash
# Round-2 GPU pass AF: shared-SIMD producer with part of each left shift done by a v_mul_f32 on a
# denormal bit pattern (tools/gen_producer.py --mulf: 2,348 vs 2,739 instructions per block).
# Parity of the experiment library on the skews tests, then C4 shard alternating product / mulf.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
EXP=tools/exp/libs3hash_mulf.so
for v in mulf mulf3; do S3H_LIBRARY=tools/exp/libs3hash_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_parity.py -k "skews" > gpurun_out/af_pytest_$v.txt 2>&1 || { tail -30 gpurun_out/af_pytest_$v.txt; exit 1; }; tail -1 gpurun_out/af_pytest_$v.txt; done
for i in 1 2; do  # variants: prod mulf mulf3
  for v in prod mulf mulf3; do
    if [ $v = prod ]; then L=s3client_amd/lib/libs3hash.so; else L=tools/exp/libs3hash_$v.so; fi
    S3H_LIBRARY=$L timeout -k 10 300 python bench.py --config c4 --kernel skews --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_af_${v}_$i.jsonl 2> gpurun_out/bench_af_${v}_$i.err || { tail -5 gpurun_out/bench_af_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/bench_af_${v}_$i.jsonl').read().strip().splitlines()[-1]); print('$v', d['value'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
  done
done
