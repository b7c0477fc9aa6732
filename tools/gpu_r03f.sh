set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/r03f
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_input_grads.py -m gpu -q -x --timeout 180 --timeout-method thread > gpurun_out/r03f/pytest.log 2>&1 || { tail -20 gpurun_out/r03f/pytest.log; exit 1; }
tail -1 gpurun_out/r03f/pytest.log
bash tools/gpu_bench_multi.sh 2 libceo_tt_base.so libceo_tt_ld4.so || exit 1
bash tools/gpu_stamps.sh
