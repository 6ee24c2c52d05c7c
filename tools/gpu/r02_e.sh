#!/bin/bash
# Round-2 GPU pass E: flag-synchronised groups -- the two-group skew kernel (2,049-4,096
# parts, C3) and the SHA-256 + MD5 group kernel (skewp range, C4 dual digest).  Full GPU
# suite first; then C3, dual C4 / C2 benches; 2-rank shared-GPU rehearsal incl. C4.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu_e.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu_e.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|error" gpurun_out/pytest_gpu_e.log | head -20; exit 1; }
B="--no-cpu-baseline --no-host-resident"
timeout -k 10 200 python bench.py $B --config c3 --steps 2 --warmup 1 > gpurun_out/e_c3.jsonl 2> gpurun_out/e_c3.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/e_c3.jsonl').read().strip().splitlines()[-1]); i=d['issue']; print('C3', d['config']['kernel'], 'grid', d['config']['grid'], 'GiB/s', d['value'], 'cyc/blk', i['cycles_per_block'], 'cpi', i['cycles_per_instr'], 'frac', i['frac'], 'bad', d['parity']['mismatches'])"
for cfg in c4 c2; do
  timeout -k 10 200 python bench.py --mode dual --config $cfg --steps 3 > gpurun_out/e_dual_$cfg.jsonl 2> gpurun_out/e_dual_$cfg.err || exit 1
  cat gpurun_out/e_dual_$cfg.jsonl
done
timeout -k 10 200 python bench.py $B --config c4 --steps 3 --warmup 1 > gpurun_out/e_c4.jsonl 2> gpurun_out/e_c4.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/e_c4.jsonl').read().strip().splitlines()[-1]); i=d['issue']; print('C4', d['config']['kernel'], 'GiB/s', d['value'], 'cyc/blk', i['cycles_per_block'], 'frac', i['frac'])"
S3H_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/e_n2_rehearsal.jsonl 2> gpurun_out/e_n2_rehearsal.err || { tail -20 gpurun_out/e_n2_rehearsal.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/e_n2_rehearsal.jsonl').read().strip().splitlines()[-1]); print('N2 rehearsal value', d['value'], 'c4', json.dumps(d.get('c4')))"
