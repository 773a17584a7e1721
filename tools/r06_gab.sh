# GPU box: group-rehash tests, then the config-4 group time of the build against a variant (abx/lib$2.so), twice.
# Usage: bash tools/r06_gab.sh TAG VARIANT
set -o pipefail
tag=${1:-x}; var=${2:-LGOLD}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_geometries.py "tests/test_gpu_scale.py" -k "group or mailbox or config4 or fused" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_gtests.log 2>&1 || { tail -40 gpurun_out/${tag}_gtests.log; exit 1; }
tail -2 gpurun_out/${tag}_gtests.log
for v in $var new $var new; do
  if [ $v = new ]; then unset ST_LIB; else export ST_LIB=$(pwd)/abx/lib$v.so; fi
  timeout -k 10 300 python3 tools/group_time.py 512 1000000 5 > gpurun_out/${tag}_gt_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_gt_$v.txt; exit 1; }
  echo "== $v $(grep group gpurun_out/${tag}_gt_$v.txt)"
done
