# Pinned staging for pageable host parts: host-path tests, app (512 MiB file) GPU vs CPU, host bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_programs.py -m gpu -x -v -k "host or dual or verify or md5 or cpp or app" --timeout 300 --timeout-method thread > gpurun_out/pytest_host_aa.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_host_aa.log; [ $rc -eq 0 ] || exit 1
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/f512.bin')" || exit 1
for jn in "8 8" "8 128"; do set -- $jn
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --verify > /dev/null 2>> gpurun_out/app_aa.log || exit 1
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 > /dev/null 2>> gpurun_out/app_aa.log || exit 1
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --cpu > /dev/null 2>> gpurun_out/app_aa.log || exit 1
done
cat gpurun_out/app_aa.log
timeout -k 10 300 python bench.py --mode host --steps 3 --warmup 1 > gpurun_out/bench_host_aa.log 2>&1 || exit 1; tail -1 gpurun_out/bench_host_aa.log
echo all ok
