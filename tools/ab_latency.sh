# Per-key latency and compare time: the in-tree build (A) against abx/libB.so (B), alternating.
set -o pipefail
for i in 1 2; do
  echo "== A"; timeout -k 10 200 python -u tools/perkey_lat.py 1000 2>&1 | tail -4 || exit 1
  echo "== B"; ST_LIB=abx/libB.so timeout -k 10 200 python -u tools/perkey_lat.py 1000 2>&1 | tail -4 || exit 1
done
echo "== A cmp"; timeout -k 10 200 python -u tools/cmp_stamps.py 2>&1 | grep "ms/compare" || exit 1
echo "== B cmp"; ST_LIB=abx/libB.so timeout -k 10 200 python -u tools/cmp_stamps.py 2>&1 | grep "ms/compare" || exit 1
