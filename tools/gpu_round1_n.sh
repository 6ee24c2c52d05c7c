# Re-entry check of the restored tree: GPU parity, smoke, default bench, rocprof stats + HBM PMC.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_n.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_n.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_n.log 2>&1 || exit 1; tail -1 gpurun_out/smoke_n.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default_n.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_n.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_quad_n -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_quad_n.log 2>&1 || exit 1
echo prof ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_quad_fetch_n -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_quad_write_n -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
echo pmc ok
