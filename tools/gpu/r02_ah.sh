#!/bin/bash
# Round-2 GPU pass AH: smoke, then the 2,188-VALU shared-SIMD producer (denormal multiplies):
# rocprofv3 kernel stats + HBM / SQ PMC for the C4 shard (skews); default bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_ah.log 2>&1 || { tail -20 gpurun_out/smoke_ah.log; exit 1; }
tail -1 gpurun_out/smoke_ah.log
B="--no-cpu-baseline --no-host-resident"
name=c4_skews
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$name -o run --output-format csv -- python3 bench.py --config c4 --steps 3 --warmup 1 $B > gpurun_out/prof_$name.jsonl 2> gpurun_out/prof_$name.err || { tail -5 gpurun_out/prof_$name.err; exit 1; }
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${name}_fetch -o run --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 0 $B > /dev/null 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${name}_write -o run --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 0 $B > /dev/null 2>&1 || exit 1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc_${name}_sq -o run --output-format csv -- python3 bench.py --config c4 --steps 2 --warmup 0 $B > /dev/null 2>&1 || exit 1
head -3 gpurun_out/prof_$name/run_kernel_stats.csv | cut -c1-160
python3 -c "import json; d=json.loads(open('gpurun_out/prof_$name.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['config']['kernel'], d['roofline']['kernel_ms'], d['issue']['cycles_per_block'], d['issue']['clock_GHz'], d['parity'])"
timeout -k 10 300 python bench.py > gpurun_out/bench_ah.jsonl 2> gpurun_out/bench_ah.err || { tail -20 gpurun_out/bench_ah.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bench_ah.jsonl').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['issue']['frac'], d['host_resident']['value'], d['cpu_baseline']['value'], d['parity'])"
