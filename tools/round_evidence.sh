#!/bin/bash
# GPU box: whole GPU suite, the default bench line (PMC traffic, CPU
# baselines, every leg), then the isolated rocprofv3 traces (timed rehash
# loop; config-4 group launch; config-5 batches).  Usage: bash tools/round_evidence.sh <tag>
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/${TAG}_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py > gpurun_out/${TAG}_bench_full.json 2> gpurun_out/${TAG}_bench_full.err || { tail -20 gpurun_out/${TAG}_bench_full.err; exit 1; }
head -c 600 gpurun_out/${TAG}_bench_full.json; echo
bash tools/trace_rehash.sh $TAG > /dev/null || exit 1
bash tools/trace_configs45.sh $TAG || exit 1
