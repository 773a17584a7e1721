# GPU box: config-5 breakdowns of the build and of variants abx/lib<V>.so (no tests: every variant computes the same
# results).  Usage: bash tools/r06_abn.sh TAG V1 V2 ...
set -o pipefail
tag=${1:-x}; shift
mkdir -p gpurun_out
for v in new "$@" new "$@"; do
  if [ $v = new ]; then unset ST_LIB; else export ST_LIB=$(pwd)/abx/lib$v.so; fi
  timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_bd_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_bd_$v.txt; exit 1; }
  echo "== $v $(grep -E 'page_merge|wall' gpurun_out/${tag}_bd_$v.txt | tr '\n' ' ')"
done
