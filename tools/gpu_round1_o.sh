# Skew kernel bring-up: parity tests for the new kernel, then C2 bench + rocprof stats.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -k "skew" --timeout 300 --timeout-method thread > gpurun_out/pytest_skew_o.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_skew_o.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --kernel skew --no-cpu-baseline > gpurun_out/bench_skew_o.log 2>&1 || exit 1; tail -1 gpurun_out/bench_skew_o.log | cut -c1-600
timeout -k 10 300 python bench.py --kernel quad --no-cpu-baseline > gpurun_out/bench_quad_o.log 2>&1 || exit 1; tail -1 gpurun_out/bench_quad_o.log | cut -c1-300
