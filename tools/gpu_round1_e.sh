set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu4.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu4.log
timeout -k 10 300 python bench.py --steps 10 --warmup 2 > gpurun_out/bench_c2_e.log 2>&1; echo "c2 rc=$?"; tail -1 gpurun_out/bench_c2_e.log | cut -c1-400
timeout -k 10 300 python bench.py --mode host --steps 3 > gpurun_out/bench_host_e.log 2>&1; echo "host rc=$?"; tail -1 gpurun_out/bench_host_e.log
timeout -k 10 600 python bench.py --config c3 --steps 2 --warmup 1 --cpu-sample-parts 32 > gpurun_out/bench_c3_e.log 2>&1; echo "c3 rc=$?"; tail -1 gpurun_out/bench_c3_e.log | cut -c1-400
for n in 16384 32768; do timeout -k 10 240 python bench.py --parts-per-gpu $n --part-bytes 262144 --kernel pair --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep2_${n}.log 2>&1; tail -1 gpurun_out/sweep2_${n}.log | cut -c1-200; done
