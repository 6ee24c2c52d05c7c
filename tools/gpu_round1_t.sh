# Lane-pair skew kernel (skewp): parity, then part-count sweep vs pair / skew.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "skewp or agree or resumable" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_t.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_t.log; [ $rc -eq 0 ] || exit 1
for np in 4096 8192 16384 32768; do for k in skewp pair; do
  timeout -k 10 120 python bench.py --kernel $k --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_t.jsonl 2>/dev/null || exit 1
done; done
timeout -k 10 120 python bench.py --kernel skew --parts-per-gpu 4096 --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_t.jsonl 2>/dev/null || exit 1
timeout -k 10 300 python bench.py --config c4 --kernel skewp --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_t.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c4_t.log | cut -c1-200
timeout -k 10 300 python bench.py --config c3 --kernel skewp --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_t.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c3_t.log | cut -c1-200
echo all ok
