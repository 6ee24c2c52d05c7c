#!/bin/bash
# Round-2 GPU pass B: rocprofv3 kernel stats + HBM / SQ PMC passes for the shipped AUTO
# kernels on C2 (skew), C4 rank-0 shard (skewp) and C3 (skew NC=2); co-issue priority
# variants; the upload app's CPU drop-in with 16 job threads (the host's CPU share).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--no-cpu-baseline --no-host-resident"
prof() {  # name, steps, bench args...
  local name=$1 steps=$2; shift 2
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python3 bench.py --steps $steps --warmup 1 $B "$@" > gpurun_out/prof_$name.jsonl 2> gpurun_out/prof_$name.err || return 1
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${name}_fetch -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${name}_write -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_${name}_sq -o run --output-format csv -- python3 bench.py --steps 2 --warmup 0 $B "$@" > /dev/null 2>&1 || return 1
  echo "prof $name done"; tail -c 400 gpurun_out/prof_$name.jsonl
}
prof c2 5 --config c2 || exit 1
prof c4 3 --config c4 || exit 1
prof c3 2 --config c3 || exit 1
timeout -k 10 120 ./tools/ubench_coissue > gpurun_out/ubench_coissue2.txt 2>&1 || exit 1
tail -6 gpurun_out/ubench_coissue2.txt
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/s3h_512.bin')"
for jn in "16 4" "16 64" "16 256"; do set -- $jn
  timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j $1 -n $2 --cpu --repeat 3 > /dev/null 2>> gpurun_out/app_cpu16.txt || exit 1
  timeout -k 10 120 ./apps/build/s3-upload-hash -f /tmp/s3h_512.bin -j $1 -n $2 --repeat 3 > /dev/null 2>> gpurun_out/app_cpu16.txt || exit 1
done
cat gpurun_out/app_cpu16.txt
rm -f /tmp/s3h_512.bin
