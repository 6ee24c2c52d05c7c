#!/bin/bash
# Round-2 GPU pass S: host-path test in the shared-SIMD kernel's range; 2-rank shared-GPU bench
# rehearsal (gloo timing collectives) whose c4 object now runs the shared-SIMD kernel.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -k "shared_simd_kernel_range" --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu_s.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu_s.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_s.log | head -20; exit 1; }
S3H_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/s_n2_rehearsal.jsonl 2> gpurun_out/s_n2_rehearsal.err || { tail -20 gpurun_out/s_n2_rehearsal.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/s_n2_rehearsal.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], json.dumps(d.get('c4'))[:600])"
