#!/bin/bash
# Round-2 GPU pass AY: MD5 experiment V2 (three LDS buffers, producer two blocks ahead, consumer
# still reads each block after its barrier: no prefetch) vs the shipped kernel, alternating;
# isolates the buffer/lead change from the prefetch measured in pass AT.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
S3H_LIBRARY=tools/exp/libs3hash_md5v2.so timeout -k 10 300 python -u -m pytest tests -m gpu -k "md5" -x -q --timeout 200 --timeout-method thread > gpurun_out/ay_pytest.txt 2>&1 || { tail -20 gpurun_out/ay_pytest.txt; exit 1; }
tail -1 gpurun_out/ay_pytest.txt
B="--no-cpu-baseline --no-host-resident --no-c5 --no-configs --steps 5 --warmup 1 --algo md5"
for i in 1 2; do for v in shipped md5v2; do
  if [ $v = shipped ]; then L=s3client_amd/lib/libs3hash.so; else L=tools/exp/libs3hash_$v.so; fi
  S3H_LIBRARY=$L timeout -k 10 200 python bench.py $B > gpurun_out/ay_${v}_$i.jsonl 2> gpurun_out/ay_${v}_$i.err || { tail -5 gpurun_out/ay_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ay_${v}_$i.jsonl').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'], d['parity'])"
done; done
