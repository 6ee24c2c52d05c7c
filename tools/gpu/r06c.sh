cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
set -o pipefail
timeout -k 10 120 python tools/pinned_range_probe.py > gpurun_out/r06c_pinned_probe.jsonl 2> gpurun_out/r06c_pinned_probe.err || exit 11
for node in 0 1; do timeout -k 10 120 tools/host_read_bw $node 16 1024 5 >> gpurun_out/r06c_host_read_bw.jsonl || exit 12; done
cat gpurun_out/r06c_host_read_bw.jsonl
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream.py -m gpu -x -v --timeout 200 --timeout-method thread -k fails_midway > gpurun_out/r06c_pytest.log 2>&1 || { tail -5 gpurun_out/r06c_pytest.log; exit 13; }
tail -1 gpurun_out/r06c_pytest.log
timeout -k 10 600 python tools/route_sweep.py --dual --reps 3 > gpurun_out/r06c_route_sweep_dual.json 2> gpurun_out/r06c_route_sweep_dual.err || { tail -5 gpurun_out/r06c_route_sweep_dual.err; exit 14; }
grep "route_sweep" gpurun_out/r06c_route_sweep_dual.err | tail -14
bash tools/gpu/power_ab.sh r06c_power 2
