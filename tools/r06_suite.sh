# GPU box: the whole GPU suite, then compare stamps and a full bench line.  Usage: bash tools/r06_suite.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 300 python3 tools/cmp_stamps.py > gpurun_out/${tag}_stamps.txt 2>&1 || { tail -20 gpurun_out/${tag}_stamps.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_stamps.txt | tail -24
timeout -k 10 600 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], 'cmp', d['compare']['ms_per_compare'], 'vu', d['verify']['verify_upper']['ms'], 'xt', d['exchange_total_ms'], 'p5', d['partition']['ms_per_batch'], d['partition']['roofline']['frac'], 'c4', d['ensembles']['ms_per_batch'], d['ensembles']['roofline']['frac'], d['ensembles'].get('kernel_trace'))"
