# Dual digest (SHA-256 + MD5 in one pass): new GPU tests, device and host-dual bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "dual or md5_host or host_path_transfer" --timeout 300 --timeout-method thread > gpurun_out/pytest_dual_v.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_dual_v.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --mode dual --steps 5 --warmup 1 > gpurun_out/bench_dual_v.log 2>&1 || exit 1; tail -1 gpurun_out/bench_dual_v.log
timeout -k 10 300 python bench.py --mode host-dual --steps 3 --warmup 1 > gpurun_out/bench_hostdual_v.log 2>&1 || exit 1; tail -1 gpurun_out/bench_hostdual_v.log
timeout -k 10 300 python bench.py --mode host --steps 3 --warmup 1 > gpurun_out/bench_host_v.log 2>&1 || exit 1; tail -1 gpurun_out/bench_host_v.log
echo all ok
