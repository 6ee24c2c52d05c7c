#!/bin/bash
# Round-2 GPU pass L: C3 solo-workgroup experiment (forced solo counts 0/22/64/128 and the
# product's model-chosen count), per-group cycles/block from the clock probe.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for v in solo0 solo22 solo64 solo128; do
  S3H_LIBRARY=tools/exp/libs3hash_$v.so timeout -k 10 240 python tools/exp_c3_solo.py --steps 3 >> gpurun_out/exp_c3_solo.jsonl 2>> gpurun_out/exp_c3_solo.err || exit 1
done
timeout -k 10 240 python tools/exp_c3_solo.py --steps 3 >> gpurun_out/exp_c3_solo.jsonl 2>> gpurun_out/exp_c3_solo.err || exit 1
cat gpurun_out/exp_c3_solo.jsonl
