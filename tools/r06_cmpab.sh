# GPU box: compare tests, then compare stamps of the build against a variant (abx/lib$2.so), twice.
# Usage: bash tools/r06_cmpab.sh TAG VARIANT
set -o pipefail
tag=${1:-x}; var=${2:-COLD}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_compare_shapes.py tests/test_gpu_parity.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py "tests/test_gpu_scale.py::test_config3_compare_10m_ordered_diff" -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for v in $var new $var new; do
  if [ $v = new ]; then unset ST_LIB; else export ST_LIB=$(pwd)/abx/lib$v.so; fi
  timeout -k 10 300 python3 tools/cmp_stamps.py > gpurun_out/${tag}_st_$v.txt 2>&1 || { tail -20 gpurun_out/${tag}_st_$v.txt; exit 1; }
  echo "== $v"; grep -E "ms/compare|stamp (verify|merge|end|placed)|slow wave" gpurun_out/${tag}_st_$v.txt | head -9
done
