#!/bin/bash
# GPU box: rocprofv3 kernel traces (--kernel-trace --stats) of the headline
# rehash (10M keys), the config-4 group rehash (512 x 1M) and config-5 paged
# batches (1M into 100M); the stats CSVs are copied to gpurun_out/<tag>_*.csv.
# Usage: bash tools/r05_prof.sh <tag>
set -o pipefail
TAG=${1:-r05}
R=$(pwd)
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $OUT/rehash -o run -- python3 $R/tools/rehash_stamps.py 10000000 12 > $OUT/rehash.log 2>&1 || { tail -5 $OUT/rehash.log; exit 1; }
cp $(find $OUT/rehash -name "*kernel_stats.csv" | head -1) $R/gpurun_out/${TAG}_rehash_kernel_stats.csv
echo rehash ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/group -o run -- python3 $R/tools/group_time.py 512 1000000 5 > $OUT/group.log 2>&1 || { tail -5 $OUT/group.log; exit 1; }
cp $(find $OUT/group -name "*kernel_stats.csv" | head -1) $R/gpurun_out/${TAG}_group512x1m_kernel_stats.csv
grep group $OUT/group.log
echo group ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/pages -o run -- python3 $R/tools/prof_pages.py 100000000 5 > $OUT/pages.log 2>&1 || { tail -5 $OUT/pages.log; exit 1; }
cp $(find $OUT/pages -name "*kernel_stats.csv" | head -1) $R/gpurun_out/${TAG}_config5_kernel_stats.csv
echo pages ok
