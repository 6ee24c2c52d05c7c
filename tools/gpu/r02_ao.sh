#!/bin/bash
# Round-2 GPU pass AO: per-device pool of host-path contexts (concurrent callers reuse theirs),
# copy threads split between concurrent calls, file slices >= 32 KiB -- host + C++ program GPU
# tests, the app's per-job mode (16 jobs) hash-only with the host trace, and config 5 again.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_cpp_programs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/ao_pytest.txt 2>&1 || { tail -30 gpurun_out/ao_pytest.txt; exit 1; }
tail -1 gpurun_out/ao_pytest.txt
python -c "import numpy as np; r=np.random.default_rng(1); f=open('/tmp/s3h_4g.bin','wb'); [f.write(r.integers(0,256,256<<20,dtype=np.uint8).tobytes()) for _ in range(16)]; f.close(); open('/tmp/s3h_512.bin','wb').write(np.random.default_rng(2).integers(0,256,512<<20,dtype=np.uint8).tobytes())"
: > gpurun_out/ao_app.txt
for src in file memory; do for pj in "" "--per-job"; do export S3H_TRACE_HOST=$([ -n "$pj" ] && echo 1 || echo 0);
  timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_4g.bin -j 16 -n 32 --source $src $pj --repeat 4 > /dev/null 2>> gpurun_out/ao_app.txt || { tail -5 gpurun_out/ao_app.txt; exit 1; }
done; done
timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_4g.bin -j 16 -n 32 --cpu --repeat 4 > /dev/null 2>> gpurun_out/ao_app.txt || exit 1
grep -v "^\[s3h host\]" gpurun_out/ao_app.txt; grep -c "^\[s3h host\]" gpurun_out/ao_app.txt || true
unset S3H_TRACE_HOST; C5_SERVER_LOG=gpurun_out/ao_server_4g.err timeout -k 10 400 python tools/c5_loopback.py /tmp/s3h_4g.bin 16 32 3 > gpurun_out/ao_c5_4g.jsonl || { cut -c1-300 gpurun_out/ao_c5_4g.jsonl; exit 1; }
C5_SERVER_LOG=gpurun_out/ao_server_512m.err timeout -k 10 300 python tools/c5_loopback.py /tmp/s3h_512.bin 16 64 3 > gpurun_out/ao_c5_512m.jsonl || { cut -c1-300 gpurun_out/ao_c5_512m.jsonl; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/ao_c5_4g.jsonl','gpurun_out/ao_c5_512m.jsonl'):
    for l in open(f):
        d=json.loads(l); print(f.split('_')[-1], d['variant'], d['parts'], d['seconds'], d['GiBps'], d['server_totals']['bad_hash'], d['server_totals']['bad_signature'])
"
