# GPU box: the whole GPU suite on the in-tree build, then bench lines (no PMC,
# no CPU legs, no trace) of the in-tree build and of abx/libB.so alternated
# (the span MD5's joined loads for misaligned spans on / off).  Usage: bash tools/r06_joinab.sh <tag>
set -o pipefail
TAG=${1:-r06ax}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 400 python3 bench.py --no-cpu --no-pmc --no-trace > gpurun_out/${TAG}_A$r.json 2> gpurun_out/${TAG}_A$r.err || exit 1
  ST_LIB=$PWD/abx/libB.so timeout -k 10 400 python3 bench.py --no-cpu --no-pmc --no-trace > gpurun_out/${TAG}_B$r.json 2> gpurun_out/${TAG}_B$r.err || exit 1
  echo "round $r done"
done
