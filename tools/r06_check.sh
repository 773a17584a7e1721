# GPU box: selected GPU tests (args) + a no-extras bench line.  Usage: bash tools/r06_check.sh TAG tests...
set -o pipefail
tag=${1:-x}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -40 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
