# GPU box: paged tests, config-5 A/B against abx/libHSINGLE.so, then the K1 MD5-form A/B (abx/libK1LAT.so).
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_paged_stream.py tests/test_int64_runs.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06am_tests.log 2>&1 || { tail -30 gpurun_out/r06am_tests.log; exit 1; }
tail -2 gpurun_out/r06am_tests.log
bash tools/r06_abn.sh r06am HSINGLE || exit 1
grep -H segment_hash gpurun_out/r06am_bd_*.txt
bash tools/r06_k1ab.sh r06al K1LAT
