set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu7.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/pytest_gpu7.log
timeout -k 10 300 python bench.py --algo md5 --steps 5 --warmup 1 --cpu-sample-parts 64 > gpurun_out/bench_md5.log 2>&1; echo "md5 rc=$?"; tail -1 gpurun_out/bench_md5.log | cut -c1-1500
timeout -k 10 60 tools/ubench_issue > gpurun_out/ubench_issue.log 2>&1; timeout -k 10 60 tools/ubench_round > gpurun_out/ubench_round.log 2>&1; echo ub $?
