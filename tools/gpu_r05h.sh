# segment lookup table: parity, then A/B against the previous build (base)
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/r05h; mkdir -p $D
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_defer.py tests/test_gpu_deterministic.py tests/test_gpu_kinks.py tests/test_gpu_peer_exchange.py -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
bash tools/gpu_bench_multi.sh 3 libceo_tt_base.so libceo_tt.so
STEPS=20 WARMUP=5 BENCH_ARGS=--no-extras bash tools/gpu_env_ab.sh 3 "BENCH=bench_prev.py CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_base.so" "CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_base.so" -
