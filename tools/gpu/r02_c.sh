#!/bin/bash
# Round-2 GPU pass C: why does skew NC=2 (C3) issue at 4.23 cycles/instr vs 4.06 for NC=1?
# Experiment builds (tools/exp, `make exp`): NC=2 with 4-block producer steps (smaller code),
# NC=2 with the producer's two items rolled, NC=1 forced on C3 (512 WGs), NC=2 forced on C2.
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-host-resident --steps 2 --warmup 1"
run() {  # tag lib config
  S3H_LIBRARY=$2 timeout -k 10 200 python bench.py $B --config $3 --kernel skew > gpurun_out/c_$1.jsonl 2> gpurun_out/c_$1.err || return 1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/c_$1.jsonl').read().strip().splitlines()[-1]); i=d['issue']; print('$1', d['config']['workload'][:30], 'grid', d['config']['grid'], 'GiB/s', d['value'], 'cyc/blk', i['cycles_per_block'], 'cpi', i['cycles_per_instr'], 'bad', d['parity']['mismatches'])"
}
run c3_default s3client_amd/lib/libs3hash.so c3 || exit 1
run c3_nc2bps4 tools/exp/libs3hash_nc2bps4.so c3 || exit 1
run c3_nc2rolled tools/exp/libs3hash_nc2rolled.so c3 || exit 1
run c3_forcenc1 tools/exp/libs3hash_forcenc1.so c3 || exit 1
run c2_default s3client_amd/lib/libs3hash.so c2 || exit 1
run c2_forcenc2 tools/exp/libs3hash_forcenc2.so c2 || exit 1
