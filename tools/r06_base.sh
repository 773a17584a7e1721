set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/part_breakdown.py 100000000 20 > gpurun_out/r06a_breakdown.txt 2>&1 || { tail -5 gpurun_out/r06a_breakdown.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/r06a_breakdown.txt | tail -40
timeout -k 10 400 python -u bench.py --no-pmc --no-cpu > gpurun_out/r06a_bench.json 2> gpurun_out/r06a_bench.err || { tail -20 gpurun_out/r06a_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r06a_bench.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['compare']['ms_per_compare'], d['partition']['ms_per_batch'], d['ensembles']['ms_per_batch'])"
