# GPU box: the default bench line (all legs, PMC and CPU baseline included).  Usage: bash tools/r06_bench.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -20 gpurun_out/${tag}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], 'cmp', d['compare']['ms_per_compare'], 'vu', d['verify']['verify_upper']['ms'], 'xt', d['exchange_total_ms'], 'p5', d['partition']['ms_per_batch'], d['partition']['roofline']['frac'], 'c4', d['ensembles']['ms_per_batch'], d['ensembles']['roofline']['frac'], d['ensembles'].get('kernel_trace'))"
