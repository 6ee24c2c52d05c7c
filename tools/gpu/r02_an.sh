#!/bin/bash
# Round-2 GPU pass AN: config 5 on loopback -- the app's --send path against the verifying mock
# S3 endpoint (GPU tests), then tools/c5_loopback.py on a 4 GiB file (16 jobs x 32 parts of
# 8 MiB) and a 512 MiB file (16 jobs x 64 parts).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_cpp_programs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/an_pytest.txt 2>&1 || { tail -30 gpurun_out/an_pytest.txt; exit 1; }
tail -1 gpurun_out/an_pytest.txt
python -c "import numpy as np; r=np.random.default_rng(1); f=open('/tmp/s3h_4g.bin','wb'); [f.write(r.integers(0,256,256<<20,dtype=np.uint8).tobytes()) for _ in range(16)]; f.close(); open('/tmp/s3h_512.bin','wb').write(np.random.default_rng(2).integers(0,256,512<<20,dtype=np.uint8).tobytes())"
timeout -k 10 400 python tools/c5_loopback.py /tmp/s3h_4g.bin 16 32 3 > gpurun_out/an_c5_4g.jsonl || { cat gpurun_out/an_c5_4g.jsonl | cut -c1-300; exit 1; }
timeout -k 10 300 python tools/c5_loopback.py /tmp/s3h_512.bin 16 64 3 > gpurun_out/an_c5_512m.jsonl || { cat gpurun_out/an_c5_512m.jsonl | cut -c1-300; exit 1; }
python3 -c "
import json
for f in ('gpurun_out/an_c5_4g.jsonl','gpurun_out/an_c5_512m.jsonl'):
    for l in open(f):
        d=json.loads(l); print(f.split('_')[-1], d['variant'], d['parts'], d['seconds'], d['GiBps'], d['server_totals']['bad_hash'], d['server_totals']['bad_signature'])
"
