# Kernel trace of the device dual-digest path: do the SHA-256 and MD5 kernels overlap?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_dual_w -o dual -- python bench.py --mode dual --steps 2 --warmup 1 > gpurun_out/prof_dual_w.log 2>&1 || exit 1
tail -1 gpurun_out/prof_dual_w.log
f=$(find gpurun_out/prof_dual_w -name '*kernel_trace.csv' | head -1); python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if "sha256" in n or "md5" in n:
        print(n[:40], r.get("Queue_Id", "?"), r.get("Stream_Id", "?"), int(r["Start_Timestamp"]) // 1000, int(r["End_Timestamp"]) // 1000, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, "ms")
PY
