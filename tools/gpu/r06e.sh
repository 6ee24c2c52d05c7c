cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
set -o pipefail
timeout -k 10 120 tools/cpu_dual_probe > gpurun_out/r06e_cpu_dual_probe.json || exit 11
cat gpurun_out/r06e_cpu_dual_probe.json
timeout -k 10 300 python tools/cpu_route_context_probe.py > gpurun_out/r06e_ctx_probe.json 2> gpurun_out/r06e_ctx_probe.err || { tail -5 gpurun_out/r06e_ctx_probe.err; exit 12; }
grep "\[ctx\]" gpurun_out/r06e_ctx_probe.err
timeout -k 10 600 python tools/route_sweep.py --dual --reps 5 > gpurun_out/r06e_route_sweep_dual.json 2> gpurun_out/r06e_route_sweep_dual.err || { tail -5 gpurun_out/r06e_route_sweep_dual.err; exit 14; }
grep "route_sweep" gpurun_out/r06e_route_sweep_dual.err | tail -16
timeout -k 10 900 python bench.py > gpurun_out/r06e_bench.jsonl 2> gpurun_out/r06e_bench.err || { tail -20 gpurun_out/r06e_bench.err; exit 15; }
tail -c 3000 gpurun_out/r06e_bench.jsonl
