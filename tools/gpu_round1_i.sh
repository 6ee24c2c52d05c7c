set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k host > gpurun_out/pytest_gpu6.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu6.log
for sl in 262144 524288 1048576 2097152; do
timeout -k 10 300 python bench.py --mode host --steps 3 --slice-bytes $sl > gpurun_out/host2_$sl.log 2>&1 || { echo "fail $sl"; break; }; tail -1 gpurun_out/host2_$sl.log | cut -c1-300
done
