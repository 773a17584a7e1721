#!/bin/bash
# GPU box: per-key and compare latency after a code change -- the per-key,
# compare and parity tests, the per-key kernel's stamps, the compare's
# stamps, per-key latency through the C-ABI and a bench line.
# Usage: bash tools/latency_checks.sh <tag>
set -o pipefail
TAG=${1:-r04}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_small_path.py tests/test_compare_shapes.py tests/test_gpu_parity.py tests/test_exchange_apply.py tests/test_concurrent_trees.py tests/test_term_keys.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_lat_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_lat_tests.log; [ $rc -eq 0 ] || exit $rc
ST_SMALL_STAMPS=1 timeout -k 10 120 python -u tools/small_stamps.py > gpurun_out/${TAG}_small_stamps.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/cmp_stamps.py > gpurun_out/${TAG}_cmp_stamps.txt 2>&1 || exit 1
timeout -k 10 200 python -u tools/perkey_lat.py > gpurun_out/${TAG}_perkey_latency.txt 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --no-cpu --no-pmc --no-cold --part-batches 2 > gpurun_out/${TAG}_bench_q.json 2> gpurun_out/${TAG}_bench_q.err || exit 1
grep -E "stamp (merge|end)|ms/compare" gpurun_out/${TAG}_cmp_stamps.txt | tail -3
tail -4 gpurun_out/${TAG}_perkey_latency.txt
python3 -c "import json;d=json.loads(open('gpurun_out/${TAG}_bench_q.json').read().strip().splitlines()[-1]);c=d['compare'];print('rehash', d['ms_per_step'], 'compare', c['ms_per_compare'], c['kernel_ms_per_compare'], 'perkey', d['ensembles']['per_key_multi']['ms_per_launch_median'], d['ensembles']['per_key_multi']['single_tree_insert1_us_median'])"
