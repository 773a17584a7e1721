#!/bin/bash
# GPU box: full GPU test suite, then a rehash-only bench line (no extras).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-extras --no-cpu --no-pmc > gpurun_out/bench_q.json 2> gpurun_out/bench_q.err || { echo "bench failed"; tail -20 gpurun_out/bench_q.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/bench_q.json')); print(d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
