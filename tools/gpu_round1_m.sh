set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_m.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu_m.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_default_m.log 2>&1 || exit 1; tail -1 gpurun_out/bench_default_m.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_quad -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_quad.log 2>&1 || exit 1
echo prof ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_quad_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_quad_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_quad_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 || exit 1
echo pmc ok
find gpurun_out/prof_quad gpurun_out/pmc_quad_fetch -name "*.csv" | head
