set -o pipefail
for v in 384 768 1536 3072; do
  echo "per_chain $v"
  S3H_GROUP_COPY_PER_CHAIN=$v timeout -k 10 300 python tools/host_small_parts.py --reps 5 || exit 1
done
