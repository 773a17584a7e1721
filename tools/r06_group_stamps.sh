# GPU box: config-4 group launch time, then its per-window phase stamps (ST_LEVEL_STAMPS=1).
# Usage: bash tools/r06_group_stamps.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/group_time.py 512 1000000 5 > gpurun_out/${tag}_group_time.txt 2>&1 || { tail -5 gpurun_out/${tag}_group_time.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_group_time.txt | tail -2
ST_LEVEL_STAMPS=1 timeout -k 10 300 python3 tools/group_time.py 512 1000000 1 > gpurun_out/${tag}_group_stamps.txt 2>&1 || { tail -5 gpurun_out/${tag}_group_stamps.txt; exit 1; }
grep -E "fused|group" gpurun_out/${tag}_group_stamps.txt | tail -40
