# GPU box: paged tests, then the config-5 breakdown of the build against a variant (abx/lib$2.so), twice.
# Usage: bash tools/r06_ab.sh TAG VARIANT
set -o pipefail
tag=${1:-x}; var=${2:-HOLD}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_ingest_small_batches.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_ptests.log 2>&1 || { tail -40 gpurun_out/${tag}_ptests.log; exit 1; }
tail -2 gpurun_out/${tag}_ptests.log
for v in $var new $var new; do
  if [ $v = new ]; then unset ST_LIB; else export ST_LIB=$(pwd)/abx/lib$v.so; fi
  timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_bd_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_bd_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${tag}_bd_$v.txt | tail -17
done
