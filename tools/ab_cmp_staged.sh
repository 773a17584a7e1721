#!/bin/bash
# GPU box: the compare's staged first pair (ST_CMP_STAGED=1) against the
# default: the compare parity tests with it on, then the per-wave stamps and
# the kernel times of both.  Usage: bash tools/ab_cmp_staged.sh <tag>
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
ST_CMP_STAGED=1 timeout -k 10 400 python -u -m pytest tests/test_compare_shapes.py tests/test_gpu_parity.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py tests/test_term_keys.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_cmp_staged_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_cmp_staged_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/cmp_stamps.py > gpurun_out/${TAG}_cmp_stamps_default.txt 2>&1 || exit 1
ST_CMP_STAGED=1 timeout -k 10 200 python -u tools/cmp_stamps.py > gpurun_out/${TAG}_cmp_stamps_staged.txt 2>&1 || exit 1
grep -E "ms/compare|stamp (merge|end)" gpurun_out/${TAG}_cmp_stamps_default.txt | tail -3
grep -E "ms/compare|stamp (merge|end)" gpurun_out/${TAG}_cmp_stamps_staged.txt | tail -3
ST_CMP_STAGED=1 timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --no-cold --part-batches 2 > gpurun_out/${TAG}_bench_cmp_staged.json 2> gpurun_out/${TAG}_bench_cmp_staged.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench_cmp_staged.json').read().strip().splitlines()[-1]);c=d['compare'];print('staged', c['ms_per_compare'], c['kernel_ms_per_compare'])"
