#!/bin/bash
# Round-2 GPU pass AS: 2-rank rehearsal of the multi-GPU bench at HEAD (both ranks on the one
# GPU, gloo for the timing collectives): C2 line + c4 object, fixture parity on both ranks.
set -o pipefail
mkdir -p gpurun_out
S3H_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/as_n2_rehearsal.jsonl 2> gpurun_out/as_n2_rehearsal.err || { tail -20 gpurun_out/as_n2_rehearsal.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/as_n2_rehearsal.jsonl').read().strip().splitlines()[-1]); print(d['n_gpus'], d['value'], d['parity'], json.dumps(d['c4']))"
