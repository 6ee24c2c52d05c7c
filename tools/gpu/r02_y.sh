#!/bin/bash
# Round-2 GPU pass Y: dual digest on C3 / C4 shard with config-correct fixtures (group kernel).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
run() {  # tag, args
  local tag=$1; shift
  timeout -k 10 400 python bench.py --mode dual --steps 2 --warmup 1 "$@" > gpurun_out/bench_y_$tag.jsonl 2> gpurun_out/bench_y_$tag.err || { tail -20 gpurun_out/bench_y_$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bench_y_$tag.jsonl').read().strip().splitlines()[-1]); print('$tag', d['value'], d['ms_per_batch'], d['fixture_mismatches'])"
}
run c3 --config c3
run c4 --config c4
run c2 --config c2
