#!/bin/bash
# Round-2 GPU pass R: LDS block padding (product: 128 B per skew block) vs none, and the LDS-pipe
# byte swap on the padded layout; C4 shard with skews, interleaved; C2 with the padded layout.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r.log 2>&1 || { tail -20 gpurun_out/smoke_r.log; exit 1; }
tail -1 gpurun_out/smoke_r.log
run() {  # tag, lib, config
  S3H_LIBRARY=$2 timeout -k 10 300 python bench.py --config $3 --steps 3 --warmup 1 --no-cpu-baseline --no-host-resident > gpurun_out/bench_r_$1.jsonl 2> gpurun_out/bench_r_$1.err || { tail -20 gpurun_out/bench_r_$1.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_r_$1.jsonl').read().strip().splitlines()[-1]); print('$1', d['config']['kernel'], d['value'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['cycles_per_instr'], d['issue']['clock_GHz'], d['parity'])"
}
run pad8_a s3client_amd/lib/libs3hash.so c4
run pad0_a tools/exp/libs3hash_pad0.so c4
run ldsbs_a tools/exp/libs3hash_ldsbswap_pad.so c4
run pad8_b s3client_amd/lib/libs3hash.so c4
run pad0_b tools/exp/libs3hash_pad0.so c4
run ldsbs_b tools/exp/libs3hash_ldsbswap_pad.so c4
run c2_pad8 s3client_amd/lib/libs3hash.so c2
