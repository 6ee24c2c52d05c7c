# Full GPU suite + smoke with skewp in AUTO; boundary sweep skewp vs pair; C4 AUTO bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_u.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_u.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_u.log 2>&1 || exit 1; tail -1 gpurun_out/smoke_u.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default_u.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_u.log | cut -c1-200
for np in 20480 24576 28672; do for k in skewp pair; do
  timeout -k 10 120 python bench.py --kernel $k --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_u.jsonl 2>/dev/null || exit 1
done; done
timeout -k 10 300 python bench.py --config c4 --steps 3 --warmup 1 > gpurun_out/bench_c4_u.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c4_u.log | cut -c1-300
echo all ok
