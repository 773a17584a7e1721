# GPU box: headline rehash (bench --no-extras) and the config-4 group time of the build against a variant, twice.
# Usage: bash tools/r06_k1ab.sh TAG VARIANT
set -o pipefail
tag=${1:-x}; var=${2:-K1LAT}
mkdir -p gpurun_out
for v in $var new $var new; do
  if [ $v = new ]; then unset ST_LIB; else export ST_LIB=$(pwd)/abx/lib$v.so; fi
  timeout -k 10 300 python3 bench.py --no-extras --no-cpu --no-pmc --no-cold --no-trace > gpurun_out/${tag}_b_$v.json 2> gpurun_out/${tag}_b_$v.err || { tail -5 gpurun_out/${tag}_b_$v.err; exit 1; }
  timeout -k 10 300 python3 tools/group_time.py 512 1000000 5 > gpurun_out/${tag}_gt_$v.txt 2>&1 || { tail -5 gpurun_out/${tag}_gt_$v.txt; exit 1; }
  echo "== $v $(python3 -c "import json; d=json.load(open('gpurun_out/${tag}_b_$v.json')); print(d['ms_per_step'], d['roofline']['kernel_avg_ms'])") $(grep group gpurun_out/${tag}_gt_$v.txt)"
done
