# GPU box: group-rehash tests, then the config-4 group launch time and its stamps.  Usage: bash tools/r06_group.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_fused_geometries.py "tests/test_gpu_scale.py" -k "group or mailbox or config4 or fused" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_gtests.log 2>&1 || { tail -40 gpurun_out/${tag}_gtests.log; exit 1; }
tail -2 gpurun_out/${tag}_gtests.log
bash tools/r06_group_stamps.sh $tag
