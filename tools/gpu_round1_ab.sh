# Host-path phase trace for the app (pageable mmap parts).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export S3H_TRACE_HOST=1
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/f512.bin')" || exit 1
for jn in "8 8" "8 128" "8 128"; do set -- $jn
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 > /dev/null 2>> gpurun_out/app_ab.log || exit 1
done
cat gpurun_out/app_ab.log
