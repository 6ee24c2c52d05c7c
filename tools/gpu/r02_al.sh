#!/bin/bash
# Round-2 GPU pass AL: file-range sources A/B on one box (tools/ab_file_parts.py), 512 MiB file,
# 1,024 / 4,096 / 8,192 parts, alternating variants, median of 15.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/s3h_512.bin')"
: > gpurun_out/al_ab.jsonl
for rep in 1 2; do for n in 1024 4096 8192; do
  PYTHONPATH=. timeout -k 10 200 python tools/ab_file_parts.py /tmp/s3h_512.bin $n 15 >> gpurun_out/al_ab.jsonl || exit 1
done; done
cat gpurun_out/al_ab.jsonl
