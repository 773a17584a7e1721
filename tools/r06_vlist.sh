# GPU box: verify-over-list A/B.  Usage: bash tools/r06_vlist.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_ingest_small_batches.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_ptests.log 2>&1 || { tail -40 gpurun_out/${tag}_ptests.log; exit 1; }
tail -2 gpurun_out/${tag}_ptests.log
for v in base list base list; do
  if [ $v = base ]; then export ST_LIB=$(pwd)/abx/libVALL.so; else unset ST_LIB; fi
  timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/${tag}_bd_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_bd_$v.txt; exit 1; }
  echo "== $v"; grep -v amdgpu.ids gpurun_out/${tag}_bd_$v.txt | tail -14
done
unset ST_LIB
bash tools/r06_trace5.sh $tag
