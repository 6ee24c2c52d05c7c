#!/bin/bash
# Round-2 GPU pass AP: one host context per device again (the device queue serialises
# batches) -- host + C++ program GPU tests and the app's per-job mode.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_cpp_programs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ap_pytest.txt 2>&1 || { tail -30 gpurun_out/ap_pytest.txt; exit 1; }
tail -1 gpurun_out/ap_pytest.txt
python -c "import numpy as np; r=np.random.default_rng(1); f=open('/tmp/s3h_4g.bin','wb'); [f.write(r.integers(0,256,256<<20,dtype=np.uint8).tobytes()) for _ in range(16)]; f.close()"
: > gpurun_out/ap_app.txt
for src in file memory; do for pj in "" "--per-job"; do
  timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_4g.bin -j 16 -n 32 --source $src $pj --repeat 4 > /dev/null 2>> gpurun_out/ap_app.txt || { tail -5 gpurun_out/ap_app.txt; exit 1; }
done; done
cat gpurun_out/ap_app.txt
