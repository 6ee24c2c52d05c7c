set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pair -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof_pair.log 2>&1 && echo prof ok
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_pair_fetch -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 && echo f ok
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_pair_write -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 && echo w ok
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_pair_sq -o run --output-format csv -- python bench.py --steps 2 --warmup 0 --no-cpu-baseline > /dev/null 2>&1 && echo sq ok
for n in 16384 32768 65536 131072; do
  for k in pair pc lane; do
    timeout -k 10 240 python bench.py --parts-per-gpu $n --part-bytes 262144 --kernel $k --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/sweep_${n}_${k}.log 2>&1 || { echo "sweep $n $k failed"; break 2; }
    python -c "import json,sys;d=json.loads(open('gpurun_out/sweep_${n}_${k}.log').read().strip().splitlines()[-1]);print('$n','$k',d['value'],d['roofline']['kernel_ms'])"
  done
done
