# GPU box: rocprofv3 kernel trace (--stats) of config-5 paged batches.  Usage: bash tools/r06_trace5.sh TAG
set -o pipefail
TAG=${1:-x}
R=$(pwd)
OUT=$R/gpurun_out/trace5_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats -f csv -d $OUT -o run -- python3 $R/tools/prof_pages.py 100000000 8 > $OUT/trace.log 2>&1 || { tail -5 $OUT/trace.log; exit 1; }
f=$(find $OUT -name "*kernel_stats.csv" | head -1)
python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:28]:
    print('%-60s %6s %10.1f us avg %8.3f ms tot' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))
"
