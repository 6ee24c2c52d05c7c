set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -x -q > gpurun_out/pytest_gpu9.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu9.log
for r in 1 2; do timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_l_$r.log 2>&1; python -c "import json;d=json.loads(open('gpurun_out/bench_l_$r.log').read().strip().splitlines()[-1]);print(d['value'],d['issue']['cycles_per_block'],d['parity'])"; done
