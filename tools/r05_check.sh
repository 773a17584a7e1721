#!/bin/bash
# GPU box: whole GPU suite, the per-key latency, the compare stamps and a
# headline-only bench line.  Usage: bash tools/r05_check.sh <tag>
set -o pipefail
TAG=${1:-r05a}
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/perkey_lat.py 2000 > gpurun_out/${TAG}_perkey_latency.txt 2>&1 || exit 1
tail -4 gpurun_out/${TAG}_perkey_latency.txt
ST_CMP_STAMPS=1 timeout -k 10 200 python -u tools/cmp_stamps.py > gpurun_out/${TAG}_cmp_stamps.txt 2>&1 || exit 1
tail -12 gpurun_out/${TAG}_cmp_stamps.txt
timeout -k 10 300 python -u bench.py --no-cpu --no-pmc --part-batches 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
head -c 400 gpurun_out/${TAG}_bench.json; echo
