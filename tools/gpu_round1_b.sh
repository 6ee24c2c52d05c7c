set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu2.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu2.log
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --cpu-sample-parts 64 > gpurun_out/bench_c4_pc.log 2>&1; echo "c4 rc=$?"
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --kernel lane --no-cpu-baseline > gpurun_out/bench_c4_lane.log 2>&1; echo "c4 lane rc=$?"
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample-parts 32 > gpurun_out/bench_c3.log 2>&1; echo "c3 rc=$?"
timeout -k 10 300 python bench.py --mode host --steps 2 > gpurun_out/bench_host.log 2>&1; echo "host rc=$?"
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/f512.bin')"
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j 8 -n 8 --verify > /dev/null 2> gpurun_out/app_gpu.log; echo "app rc=$?"
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j 8 -n 8 --cpu > /dev/null 2> gpurun_out/app_cpu.log; echo "appcpu rc=$?"
for f in bench_c4_pc bench_c4_lane bench_c3 bench_host app_gpu app_cpu; do echo "== $f"; tail -2 gpurun_out/$f.log | cut -c1-1500; done
