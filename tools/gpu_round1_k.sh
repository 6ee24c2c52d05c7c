set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu8.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu8.log
for a in md5 sha256; do timeout -k 10 300 python bench.py --algo $a --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k_$a.log 2>&1; echo "$a rc=$?"; python -c "import json;d=json.loads(open('gpurun_out/bench_k_$a.log').read().strip().splitlines()[-1]);print(d['value'],d['issue'],d['parity'])"; done
timeout -k 10 300 python bench.py --kernel pc --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k_pc.log 2>&1; python -c "import json;d=json.loads(open('gpurun_out/bench_k_pc.log').read().strip().splitlines()[-1]);print('pc',d['value'],d['issue']['cycles_per_block'])"
timeout -k 10 300 python bench.py --kernel lane --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/bench_k_lane.log 2>&1; python -c "import json;d=json.loads(open('gpurun_out/bench_k_lane.log').read().strip().splitlines()[-1]);print('lane',d['value'],d['issue']['cycles_per_block'])"
