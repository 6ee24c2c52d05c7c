#!/bin/bash
# Round-2 GPU pass A: full GPU suite (incl. full-size C3 / C4), smoke, default bench line,
# co-issue + host-registration microbenchmarks, upload-app host-path timings.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default.jsonl 2> gpurun_out/bench_default.err || exit 1
cut -c1-600 gpurun_out/bench_default.jsonl
timeout -k 10 120 ./tools/ubench_coissue > gpurun_out/ubench_coissue.txt 2>&1 || exit 1
cat gpurun_out/ubench_coissue.txt
timeout -k 10 120 ./tools/ubench_hostreg > gpurun_out/ubench_hostreg.txt 2>&1 || exit 1
cat gpurun_out/ubench_hostreg.txt
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/s3h_512.bin')"
for n in 64 1024 4096; do
  for src in file mmap memory; do
    S3H_TRACE_HOST=1 timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j 1 -n $n --source $src --repeat 3 > /dev/null 2>> gpurun_out/app_upload.txt || exit 1
  done
  timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j 1 -n $n --cpu --repeat 3 > /dev/null 2>> gpurun_out/app_upload.txt || exit 1
done
grep -v "^\[s3h host\]" gpurun_out/app_upload.txt
rm -f /tmp/s3h_512.bin
