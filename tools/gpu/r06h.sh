cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
set -o pipefail
S3H_TRACE_ROUTE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_route_adapt.py -m gpu -x -v -s --timeout 400 --timeout-method thread > gpurun_out/r06h_route_adapt.log 2>&1 || { tail -30 gpurun_out/r06h_route_adapt.log; exit 11; }
tail -1 gpurun_out/r06h_route_adapt.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread --ignore=tests/test_gpu_bench.py --ignore=tests/test_gpu_configs.py --ignore=tests/test_gpu_enomem.py --ignore=tests/test_gpu_errors.py --ignore=tests/test_gpu_host.py --ignore=tests/test_gpu_numa.py --ignore=tests/test_gpu_parity.py --ignore=tests/test_gpu_policy.py --ignore=tests/test_gpu_route_adapt.py --ignore=tests/test_buffer_parts.py --ignore=tests/test_code_object.py --ignore=tests/test_cpp_programs.py > gpurun_out/r06h_rest.log 2>&1 || { tail -30 gpurun_out/r06h_rest.log; exit 12; }
tail -1 gpurun_out/r06h_rest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06h_smoke.log 2>&1 || { tail -5 gpurun_out/r06h_smoke.log; exit 13; }
tail -1 gpurun_out/r06h_smoke.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r06h_stats_prof -o run --output-format csv -- python3 bench.py > gpurun_out/r06h_stats.jsonl 2> gpurun_out/r06h_stats.err || { tail -5 gpurun_out/r06h_stats.err; exit 14; }
python3 tools/gpu/summary.py gpurun_out/r06h_stats.jsonl
