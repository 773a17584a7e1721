#!/bin/bash
# Full bench line (every leg, no PMC / CPU legs) for the round-2 kernel and
# the progressive one, prog stamps, and the config-5 batch breakdown.
mkdir -p gpurun_out
ST_REHASH=prog ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps.py > gpurun_out/prog_stamps_p3.txt 2>&1 || exit $?
ST_REHASH=prog ST_PG_PRIO=0 ST_LEVEL_STAMPS=1 timeout -k 10 120 python3 tools/stamps.py > gpurun_out/prog_stamps_p0.txt 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/full_fused.json 2> gpurun_out/full_fused.err || exit $?
ST_REHASH=prog timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 --no-pmc --no-cpu > gpurun_out/full_prog.json 2> gpurun_out/full_prog.err || exit $?
timeout -k 10 300 python -u tools/part_breakdown.py > gpurun_out/part_bd_span.txt 2>&1 || exit $?
tail -4 gpurun_out/part_bd_span.txt
