# A/B of the fused rehash: the in-tree build against abx/libB.so, alternating.
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python3 tools/rehash_span.py 10000000 200 5 2>&1 | grep span || exit 1
  ST_LIB=abx/libB.so timeout -k 10 120 python3 tools/rehash_span.py 10000000 200 5 2>&1 | grep span || exit 1
done
