#!/bin/bash
# Round-2 GPU pass AM: 128 MiB staging slots for file ranges -- host-path GPU tests, then the
# file-source A/B (tools/ab_file_parts.py, median of 11, twice) and the app at 1,024-8,192 parts.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v --timeout 200 --timeout-method thread > gpurun_out/am_pytest.txt 2>&1 || { tail -30 gpurun_out/am_pytest.txt; exit 1; }
tail -1 gpurun_out/am_pytest.txt
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/s3h_512.bin')"
: > gpurun_out/am_ab.jsonl
for rep in 1 2; do for n in 1024 4096 8192; do
  PYTHONPATH=. timeout -k 10 200 python tools/ab_file_parts.py /tmp/s3h_512.bin $n 11 >> gpurun_out/am_ab.jsonl || exit 1
done; done
cat gpurun_out/am_ab.jsonl
: > gpurun_out/am_app.txt
for jn in "16 64" "16 128" "16 256" "16 512"; do set -- $jn
  for src in file mmap; do
    S3H_TRACE_HOST=1 timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j $1 -n $2 --source $src --repeat 5 > /dev/null 2>> gpurun_out/am_app.txt || { tail -5 gpurun_out/am_app.txt; exit 1; }
  done
done
grep "gpu batch" gpurun_out/am_app.txt
