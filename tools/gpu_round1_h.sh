set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu5.log 2>&1; echo "pytest rc=$?"; tail -3 gpurun_out/pytest_gpu5.log
for sl in 262144 524288 1048576 2097152; do
timeout -k 10 300 python bench.py --mode host --steps 3 --slice-bytes $sl > gpurun_out/host_$sl.log 2>&1 || { echo "fail $sl"; break; }; tail -1 gpurun_out/host_$sl.log
done
