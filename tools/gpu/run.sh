#!/bin/bash
# One parameterised runner for every GPU pass (replaces round 2's one-shot tools/gpu/r02_*.sh).
#
#   gpurun --timeout 1200 -- 'bash tools/gpu/run.sh TAG STEP [STEP ...]'
#
# Each STEP is NAME or NAME:ARGS (pytest ARGS are eval-ed: quote a -k expression); steps run in order, each under its own
# time limit, and the first failure ends the pass (no retries).  Outputs go to
# gpurun_out/<TAG>_<n>_<NAME>.{log,jsonl,err} and a one-line summary per step to stdout.
#   pytest[:ARGS]        python -m pytest tests -m gpu -x -v ARGS            (900 s)
#   pytestlib:LIB[:ARGS] the same against an experiment build (S3H_LIBRARY=LIB)
#   smoke                __graft_entry__.smoke()                              (120 s)
#   bench[:ARGS]         python bench.py ARGS -> one JSON line                (400 s)
#   benchlib:LIB[:ARGS]  the same with S3H_LIBRARY=LIB (a `make exp` build)    (400 s)
#   stats[:ARGS]         rocprofv3 --kernel-trace --stats of bench.py ARGS    (400 s)
#   pmc[:CTRS[:ARGS]]    rocprofv3 --pmc CTRS (one pass, e.g. FETCH_SIZE) of bench.py ARGS (240 s)
#   pmclib:LIB:CTRS[:ARGS] the same on an experiment build (S3H_LIBRARY=LIB)     (240 s)
#   n2[:ARGS]            2-rank torch.distributed.run rehearsal of bench.py on the one GPU
#                        (S3H_BENCH_SHARE_GPU=1, gloo collectives, as the driver's N>1 runs) (600 s)
#   selfn:N[:ARGS]       `python bench.py --gpus N ARGS` with NO launcher (bench.py starts the N
#                        ranks itself) on the one GPU, S3H_BENCH_SHARE_GPU=1          (600 s)
#   py:SCRIPT[:ARGS]     python SCRIPT ARGS                                  (600 s)
#   trace:SCRIPT         rocprofv3 --kernel-trace --memory-copy-trace of python3 SCRIPT (300 s)
#   exe:PROGRAM ARGS     a built tool, e.g. tools/ubench_dep                  (300 s)
#   make:ARGS            make ARGS on the box, e.g. an experiment build (tools/exp is
#                        gpurun-ignored: experiment libraries are built where they run) (600 s)
set -o pipefail
TAG=${1:?usage: run.sh TAG STEP...}; shift
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
n=0
for step in "$@"; do
  n=$((n + 1))
  name=${step%%:*}; rest=""; [ "$step" != "$name" ] && rest=${step#*:}
  out=gpurun_out/${TAG}_${n}_${name}
  case $name in
    pytest)
      eval "timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $rest" > $out.log 2>&1; rc=$?
      tail -1 $out.log ;;
    pytestlib)  # pytestlib:LIB:ARGS -- GPU tests against an experiment build (S3H_LIBRARY=LIB)
      lib=${rest%%:*}; args=""; [ "$rest" != "$lib" ] && args=${rest#*:}
      eval "S3H_LIBRARY=$lib timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread $args" > $out.log 2>&1; rc=$?
      tail -1 $out.log ;;
    smoke)
      timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $out.log 2>&1; rc=$?
      tail -1 $out.log ;;
    bench)
      timeout -k 10 400 python bench.py $rest > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && python3 tools/gpu/summary.py $out.jsonl ;;
    benchlib)  # benchlib:LIB:ARGS -- bench.py on an experiment build (S3H_LIBRARY=LIB)
      lib=${rest%%:*}; args=""; [ "$rest" != "$lib" ] && args=${rest#*:}
      S3H_LIBRARY=$lib timeout -k 10 400 python bench.py $args > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && python3 tools/gpu/summary.py $out.jsonl ;;
    stats)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d ${out}_prof -o run --output-format csv -- python3 bench.py $rest > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && head -4 ${out}_prof/run_kernel_stats.csv | cut -c1-200 ;;
    pmc)
      ctrs=${rest%%:*}; args=""; [ "$rest" != "$ctrs" ] && args=${rest#*:}
      timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d ${out}_prof -o run --output-format csv -- python3 bench.py $args > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && ls ${out}_prof ;;
    pmclib)  # pmclib:LIB:CTRS:ARGS -- one --pmc pass of bench.py on an experiment build
      lib=${rest%%:*}; r2=${rest#*:}; ctrs=${r2%%:*}; args=""; [ "$r2" != "$ctrs" ] && args=${r2#*:}
      S3H_LIBRARY=$lib timeout -s KILL 240 rocprofv3 --pmc $ctrs --kernel-trace -d ${out}_prof -o run --output-format csv -- python3 bench.py $args > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && ls ${out}_prof ;;
    n2)
      S3H_BENCH_SHARE_GPU=1 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 $rest > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && python3 tools/gpu/summary.py $out.jsonl ;;
    selfn)
      nr=${rest%%:*}; args=""; [ "$rest" != "$nr" ] && args=${rest#*:}
      S3H_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus $nr $args > $out.jsonl 2> $out.err; rc=$?
      [ $rc -eq 0 ] && python3 tools/gpu/summary.py $out.jsonl ;;
    make)
      eval "timeout -k 10 600 make -j16 $rest" > $out.log 2>&1; rc=$?
      tail -1 $out.log ;;
    exe)  # exe:PROGRAM [ARGS] -- a built tool (e.g. tools/ubench_dep), output to .log
      timeout -k 10 300 $rest > $out.log 2>&1; rc=$?
      tail -12 $out.log ;;
    trace)  # trace:SCRIPT -- kernel + memory-copy trace (no counters) of python3 SCRIPT
      timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d ${out}_prof -o run --output-format csv -- python3 $rest > $out.log 2> $out.err; rc=$?
      [ $rc -eq 0 ] && tail -2 $out.log ;;
    py)
      script=${rest%%:*}; args=""; [ "$rest" != "$script" ] && args=${rest#*:}
      timeout -k 10 600 python -u $script $args > $out.log 2>&1; rc=$?
      tail -3 $out.log ;;
    *) echo "unknown step $name"; exit 2 ;;
  esac
  if [ $rc -ne 0 ]; then
    echo "step $n ($step) failed: rc $rc"
    for f in $out.log $out.err; do [ -f $f ] && tail -25 $f; done
    exit 1
  fi
done
