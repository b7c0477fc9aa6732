set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/r05j; mkdir -p $D
timeout -k 10 600 python -u -m pytest "tests/test_gpu_peer_exchange.py::test_peer_exchange_mean_and_adam" -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_ex.log 2>&1 || { tail -30 $D/pytest_ex.log; exit 1; }
tail -1 $D/pytest_ex.log
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_both.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kinks.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_both.log 2>&1 || { tail -30 $D/pytest_both.log; exit 1; }
tail -1 $D/pytest_both.log
bash tools/gpu_bench_multi.sh 3 libceo_tt.so libceo_tt_frf.so libceo_tt_prf.so libceo_tt_both.so
