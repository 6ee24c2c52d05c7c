# Skew fast/slow loop split: full GPU suite, default bench, NC=4 skew vs pair at 8192 parts,
# C3 and C4 configs.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_q.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_q.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_default_q.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_q.log | cut -c1-250
for np in 6144 8192; do
  S3H_QUAD_WAVES=4 timeout -k 10 120 python bench.py --kernel skew --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_q.jsonl 2>/dev/null || exit 1
  timeout -k 10 120 python bench.py --kernel pair --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_q.jsonl 2>/dev/null || exit 1
done
S3H_QUAD_WAVES=4 timeout -k 10 300 python bench.py --config c4 --kernel skew --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_skew4_q.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c4_skew4_q.log | cut -c1-250
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_q.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c3_q.log | cut -c1-250
echo all ok
