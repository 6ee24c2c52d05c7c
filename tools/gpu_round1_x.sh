# Fused dual-digest kernel: tests, device + host-dual bench, kernel trace (overlap check).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k "dual or md5 or skew" --timeout 300 --timeout-method thread > gpurun_out/pytest_dual_x.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dual_x.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --mode dual --steps 5 --warmup 1 > gpurun_out/bench_dual_x.log 2>&1 || exit 1; tail -1 gpurun_out/bench_dual_x.log
timeout -k 10 300 python bench.py --mode host-dual --steps 3 --warmup 1 > gpurun_out/bench_hostdual_x.log 2>&1 || exit 1; tail -1 gpurun_out/bench_hostdual_x.log
timeout -k 10 300 python bench.py --mode dual --config c4 --steps 2 --warmup 1 > gpurun_out/bench_dual_c4_x.log 2>&1 || exit 1; tail -1 gpurun_out/bench_dual_c4_x.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dual_x -o dual -- python bench.py --mode dual --steps 3 --warmup 1 > gpurun_out/prof_dual_x.log 2>&1 || exit 1
f=$(find gpurun_out/prof_dual_x -name '*kernel_trace.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "sha256" in n or "md5" in n:
        print(n[:48], int(r["Start_Timestamp"]) // 1000, int(r["End_Timestamp"]) // 1000, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "ms")
PY
echo all ok
