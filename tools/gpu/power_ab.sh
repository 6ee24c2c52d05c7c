#!/bin/bash
# C4-shard power attribution: the product's shared-SIMD skews kernel beside
# two experiment builds of the same source -- consumers alone on stale W+K (producers keep only
# the flag protocol: make exp TAG=pidle EXPFLAGS=-DS3H_EXP_PRODUCER_IDLE) and producers alone
# (consumers keep only the flag protocol: TAG=cidle, -DS3H_EXP_CONSUMER_IDLE) -- alternated in
# one lease, each a bench.py --config c4 --kernel skews line with amdsmi board power and clock.
# The experiment builds' digests are wrong by design: their bench exits 3 (parity), accepted;
# any other failure ends the pass.
#   bash tools/gpu/power_ab.sh TAG [ROUNDS]
set -o pipefail
TAG=${1:?usage: power_ab.sh TAG [ROUNDS]}; ROUNDS=${2:-2}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
ARGS="--config c4 --kernel skews --steps 5 --warmup 2 --no-cpu-baseline"
for r in $(seq 1 "$ROUNDS"); do
  for v in product pidle cidle; do
    out=gpurun_out/${TAG}_${r}_${v}.jsonl
    lib=""
    [ "$v" != product ] && lib=tools/exp_r06/libs3hash_$v.so
    S3H_LIBRARY=${lib:-s3client_amd/lib/libs3hash.so} timeout -k 10 300 python bench.py $ARGS > $out 2> ${out%.jsonl}.err; rc=$?
    if [ $rc -ne 0 ] && ! { [ $rc -eq 3 ] && [ "$v" != product ]; }; then echo "$v round $r: rc $rc"; exit $rc; fi
    python3 - "$out" "$v" <<'PY'
import json, sys
l = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = l.get("power", {})
print(sys.argv[2], round(l["value"], 1), "GiB/s", "busy W", p.get("busy_mean_W"), "max W", p.get("max_W"),
      "MHz", p.get("busy_clock_MHz_mean"), "cyc/blk", l.get("issue", {}).get("cycles_per_block"))
PY
  done
done
