#!/bin/bash
# Round-2 GPU pass AT: MD5 producer/consumer kernel with three LDS buffers (consumer prefetches
# the next block's M+K) -- MD5 / dual / stream GPU tests, then C2 MD5 alternating with the
# previous kernel (tools/exp/libs3hash_md5old.so, HEAD~ sources), dual digest lines, and
# rocprofv3 kernel stats of the C2 MD5 line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -k "md5 or dual or etag or stream or verify" -x -v --timeout 300 --timeout-method thread > gpurun_out/at_pytest.txt 2>&1 || { tail -30 gpurun_out/at_pytest.txt; exit 1; }
tail -1 gpurun_out/at_pytest.txt
B="--no-cpu-baseline --no-host-resident --no-c5 --steps 5 --warmup 1"
for i in 1 2; do for v in new old; do
  if [ $v = new ]; then L=s3client_amd/lib/libs3hash.so; else L=tools/exp/libs3hash_md5old.so; fi
  S3H_LIBRARY=$L timeout -k 10 200 python bench.py --algo md5 $B > gpurun_out/at_md5_${v}_$i.jsonl 2> gpurun_out/at_md5_${v}_$i.err || { tail -5 gpurun_out/at_md5_${v}_$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/at_md5_${v}_$i.jsonl').read().strip().splitlines()[-1]); print('md5 c2 $v', d['value'], d['ms_per_step'], d['parity'])"
done; done
for cfg in c2 c4; do
  timeout -k 10 300 python bench.py --mode dual --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/at_dual_$cfg.jsonl 2> gpurun_out/at_dual_$cfg.err || { tail -5 gpurun_out/at_dual_$cfg.err; exit 1; }
  tail -1 gpurun_out/at_dual_$cfg.jsonl | cut -c1-400
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_md5_at -o run --output-format csv -- python3 bench.py --algo md5 $B > gpurun_out/prof_md5_at.jsonl 2> gpurun_out/prof_md5_at.err || { tail -5 gpurun_out/prof_md5_at.err; exit 1; }
head -3 gpurun_out/prof_md5_at/run_kernel_stats.csv | cut -c1-160
