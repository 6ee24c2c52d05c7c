#!/bin/bash
# Round-2 GPU pass AK: s3h_sha256_file_parts maps the file above 1,024 parts per device --
# host-path GPU tests, then the 512 MiB upload file at 1,024 / 4,096 / 8,192 parts from each
# source (file ranges, mmap, memory), 3 repeats each, with the host-phase trace.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_host.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ak_pytest.txt 2>&1 || { tail -30 gpurun_out/ak_pytest.txt; exit 1; }
tail -1 gpurun_out/ak_pytest.txt
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/s3h_512.bin')"
: > gpurun_out/ak_app.txt
for jn in "16 64" "16 128" "16 256" "16 512"; do set -- $jn
  for src in file mmap memory; do
    S3H_TRACE_HOST=1 timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j $1 -n $2 --source $src --repeat 3 > /dev/null 2>> gpurun_out/ak_app.txt || { tail -5 gpurun_out/ak_app.txt; exit 1; }
  done
done
grep "gpu batch" gpurun_out/ak_app.txt
