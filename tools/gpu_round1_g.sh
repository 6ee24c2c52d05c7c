set -o pipefail
cd $GRAFT_REPO_ROOT
for sl in 262144 524288 1048576 2097152; do
timeout -k 10 300 python bench.py --mode host --steps 3 --slice-bytes $sl > gpurun_out/host_$sl.log 2>&1 || { echo "fail $sl"; break; }; tail -1 gpurun_out/host_$sl.log
done
