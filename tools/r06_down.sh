# GPU box: the paged-merge tests (checked cases first), then the config-5
# breakdown with in-place merges never / by the bytes / always shifting down
# (st_debug_knob ST_DBG_PAGE_DOWN 0, 1, 2).  Usage: bash tools/r06_down.sh <tag>
set -o pipefail
TAG=${1:-r06as}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_paged_stream.py tests/test_int64_runs.py -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
rc=$?; tail -4 gpurun_out/${TAG}_tests.log; [ $rc -eq 0 ] || exit $rc
for m in 0 1 0 1; do
  timeout -k 10 300 python tools/part_breakdown.py 100000000 30 down$m > gpurun_out/${TAG}_bd_down$m.txt 2>&1 || exit 1
  echo "down$m: $(tail -1 gpurun_out/${TAG}_bd_down$m.txt | cut -c1-60) page_merge: $(grep page_merge gpurun_out/${TAG}_bd_down$m.txt)"
done
