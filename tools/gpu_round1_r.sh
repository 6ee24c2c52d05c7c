# Default bench (with clock probe + CPU baseline), rocprof stats + HBM/SQ PMC for the skew
# fast-loop kernel, host and stream modes.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > gpurun_out/bench_default_r.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_r.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_skew_r -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_skew_r.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_skew_fetch_r -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_skew_write_r -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_skew_sq_r -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
echo prof ok
timeout -k 10 300 python bench.py --mode host --no-cpu-baseline > gpurun_out/bench_host_r.log 2>&1 || exit 1; tail -1 gpurun_out/bench_host_r.log | cut -c1-300
timeout -k 10 300 python bench.py --mode stream --no-cpu-baseline > gpurun_out/bench_stream_r.log 2>&1 || exit 1; tail -1 gpurun_out/bench_stream_r.log | cut -c1-300
