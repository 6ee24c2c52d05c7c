# Full GPU regression of the tree after the pinned-staging host path: pytest -m gpu, smoke,
# default bench (with CPU baseline), rocprofv3 stats of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_ad.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_ad.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ad.log 2>&1 || exit 1; tail -1 gpurun_out/smoke_ad.log
timeout -k 10 400 python bench.py > gpurun_out/bench_default_ad.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_ad.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_default_ad -o c2 -- python bench.py --no-cpu-baseline > gpurun_out/prof_default_ad.log 2>&1 || exit 1
cat $(find gpurun_out/prof_default_ad -name '*kernel_stats.csv' | head -1) | head -5
echo all ok
