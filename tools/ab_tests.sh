# The paged-stream tests against the in-tree build, then the config-5 A/B.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_paged_stream.py -m gpu -q -x --timeout 120 --timeout-method thread 2>&1 | tail -15
bash tools/ab_pages.sh ${1:-abt}
