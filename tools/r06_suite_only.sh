# GPU box: the whole GPU suite, then the repair / rehash-after-mutation breakdown.  Usage: bash tools/r06_suite_only.sh TAG
set -o pipefail
tag=${1:-x}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_gpu.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest_gpu.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest_gpu.log
timeout -k 10 300 python3 tools/repair_breakdown.py > gpurun_out/${tag}_repair.txt 2>&1 || { tail -10 gpurun_out/${tag}_repair.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${tag}_repair.txt | tail -20
