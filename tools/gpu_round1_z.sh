# Upload counterpart app (config 5 offline): GPU host path vs CPU drop-in on a 512 MiB file.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
python -c "import numpy as np; np.random.default_rng(1).integers(0,256,512<<20,dtype=np.uint8).tofile('/tmp/f512.bin')" || exit 1
for jn in "8 8" "8 128"; do set -- $jn
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --verify > /dev/null 2>> gpurun_out/app_z.log || exit 1
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 > /dev/null 2>> gpurun_out/app_z.log || exit 1
timeout -k 10 120 apps/build/s3-upload-hash -f /tmp/f512.bin -j $1 -n $2 --cpu > /dev/null 2>> gpurun_out/app_z.log || exit 1
done
cat gpurun_out/app_z.log
