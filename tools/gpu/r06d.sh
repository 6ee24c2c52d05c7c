cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp PYTHONUNBUFFERED=1
set -o pipefail
timeout -k 10 120 tools/cpu_dual_probe > gpurun_out/r06d_cpu_dual_probe.json || exit 11
cat gpurun_out/r06d_cpu_dual_probe.json
timeout -k 10 60 python -c "
import time, json
import sys; sys.path.insert(0, 'tools')
from power import PowerSampler
import torch
torch.cuda.init()
import s3client_amd as s3
bdf = s3.device_pci_bus_id(0)
with PowerSampler(bdf) as pw:
    time.sleep(3)
print(json.dumps({'idle_board_power': pw.summary(), 'power_cap_W': s3.device_power_cap(0), 'bdf': bdf}))
" > gpurun_out/r06d_idle_power.json 2>&1 || { tail -3 gpurun_out/r06d_idle_power.json; exit 12; }
tail -1 gpurun_out/r06d_idle_power.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_host.py tests/test_gpu_stream.py tests/test_gpu_route_adapt.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r06d_pytest.log 2>&1 || { tail -30 gpurun_out/r06d_pytest.log; exit 13; }
tail -1 gpurun_out/r06d_pytest.log
timeout -k 10 600 python tools/route_sweep.py --dual --reps 3 > gpurun_out/r06d_route_sweep_dual.json 2> gpurun_out/r06d_route_sweep_dual.err || { tail -5 gpurun_out/r06d_route_sweep_dual.err; exit 14; }
grep "route_sweep" gpurun_out/r06d_route_sweep_dual.err | tail -16
