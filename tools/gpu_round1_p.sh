# Full GPU suite with skew as AUTO, smoke, default bench, host-path bench, skew sweep over part
# counts (NC=1/2 region and beyond), rocprof stats + HBM PMC of the default bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_p.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_p.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_p.log 2>&1 || exit 1; tail -1 gpurun_out/smoke_p.log
timeout -k 10 300 python bench.py > gpurun_out/bench_default_p.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_p.log | cut -c1-300
timeout -k 10 300 python bench.py --mode host --no-cpu-baseline > gpurun_out/bench_host_p.log 2>&1 || exit 1; tail -1 gpurun_out/bench_host_p.log | cut -c1-300
for np in 2048 4096 8192; do for k in skew quad pair; do
  timeout -k 10 120 python bench.py --kernel $k --parts-per-gpu $np --part-bytes 262144 --steps 5 --warmup 1 --no-cpu-baseline >> gpurun_out/sweep_p.jsonl 2>/dev/null || exit 1
done; done
echo sweep ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_skew_p -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_skew_p.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_skew_fetch_p -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_skew_write_p -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_skew_sq_p -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
echo prof ok
