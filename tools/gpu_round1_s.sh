# Skew producer with 8-block steps for NC = 2, 4: parity on multi-wave plans, then sweeps.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "skew or two_consumer or resumable or agree" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_s.log; [ $rc -eq 0 ] || exit 1
S3H_QUAD_WAVES=4 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "skew" --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_s4.log 2>&1; rc=$?; echo "pytest NC4 rc=$rc"; tail -3 gpurun_out/pytest_gpu_s4.log; [ $rc -eq 0 ] || exit 1
for np in 2048 4096; do
  timeout -k 10 120 python bench.py --kernel skew --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_s.jsonl 2>/dev/null || exit 1
done
for np in 6144 8192; do
  S3H_QUAD_WAVES=4 timeout -k 10 120 python bench.py --kernel skew --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_s.jsonl 2>/dev/null || exit 1
done
timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c3_s.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c3_s.log | cut -c1-200
S3H_QUAD_WAVES=4 timeout -k 10 300 python bench.py --config c4 --kernel skew --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_c4_s.log 2>&1 || exit 1; tail -1 gpurun_out/bench_c4_s.log | cut -c1-200
echo all ok
