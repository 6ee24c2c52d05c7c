#!/bin/bash
# Round-2 GPU pass D: (1) NC=2 with only consumer wave 0 working (is the NC=2 slowdown
# contention between the two consumers?); (2) 2-rank shared-GPU rehearsal of the multi-GPU
# bench (gloo for the timing collectives) incl. the C4 sub-object.
set -o pipefail
mkdir -p gpurun_out
B="--no-cpu-baseline --no-host-resident --steps 2 --warmup 1"
S3H_LIBRARY=tools/exp/libs3hash_lone2.so timeout -k 10 120 python bench.py $B --config c2 --kernel skew > gpurun_out/d_lone2.jsonl 2> gpurun_out/d_lone2.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/d_lone2.jsonl').read().strip().splitlines()[-1]); i=d['issue']; print('lone2 grid', d['config']['grid'], 'cyc/blk', i['cycles_per_block'], 'cpi', i['cycles_per_instr'], 'waves', i.get('waves'))"
S3H_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/d_n2_rehearsal.jsonl 2> gpurun_out/d_n2_rehearsal.err || { tail -20 gpurun_out/d_n2_rehearsal.err; exit 1; }
cut -c1-300 gpurun_out/d_n2_rehearsal.jsonl; python3 -c "import json; d=json.loads(open('gpurun_out/d_n2_rehearsal.jsonl').read().strip().splitlines()[-1]); print(json.dumps(d.get('c4')))"
