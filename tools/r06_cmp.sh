# GPU box: compare tests + compare stamps + a bench line.  Usage: bash tools/r06_cmp.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_compare_shapes.py tests/test_gpu_parity.py tests/test_exchange_apply.py tests/test_partitioned_exchange.py tests/test_remote_exchange.py tests/test_concurrent_trees.py "tests/test_gpu_scale.py::test_config3_compare_10m_ordered_diff" -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 300 python3 tools/cmp_stamps.py > gpurun_out/${tag}_stamps.txt 2>&1 || { tail -20 gpurun_out/${tag}_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_stamps.txt | tail -24
timeout -k 10 300 python -u bench.py --no-pmc --no-cpu --no-cold > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], 'cmp', d['compare']['ms_per_compare'], d['compare']['kernel_ms_per_compare'], 'vu', d['verify']['verify_upper']['ms'], 'xt', d['exchange_total_ms'], 'p5', d['partition']['ms_per_batch'], 'c4', d['ensembles']['ms_per_batch'])"
