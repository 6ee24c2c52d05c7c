# Host path with the buffer cache: host/app GPU tests, app steady state (512 MiB file) GPU vs
# CPU, with the host-path phase trace.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_cpp_programs.py -m gpu -x -v -k "host or dual or verify or md5 or cpp or app" --timeout 300 --timeout-method thread > gpurun_out/pytest_host_ac.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_host_ac.log; [ $rc -eq 0 ] || exit 1
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/f512.bin')" || exit 1
for jn in "8 8" "8 128" "16 256"; do set -- $jn
S3H_TRACE_HOST=1 timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --repeat 3 --verify > /dev/null 2>> gpurun_out/app_ac.log || exit 1
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --repeat 3 --cpu > /dev/null 2>> gpurun_out/app_ac.log || exit 1
done
cat gpurun_out/app_ac.log
echo all ok
