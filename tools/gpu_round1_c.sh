set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu3.log 2>&1; echo "pytest rc=$?"; tail -15 gpurun_out/pytest_gpu3.log
timeout -k 10 300 python bench.py --steps 5 --warmup 1 > gpurun_out/bench_c2_pair.log 2>&1; echo "c2 pair rc=$?"; tail -1 gpurun_out/bench_c2_pair.log | cut -c1-900
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_pair.log 2>&1; echo "c4 rc=$?"; tail -1 gpurun_out/bench_c4_pair.log | cut -c1-700
