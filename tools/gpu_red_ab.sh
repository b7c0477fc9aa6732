# parity of a reduce-shape variant, then interleaved bench: bash tools/gpu_red_ab.sh variant.so [others...]
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/red
CEO_TT_LIB=ceo-recommender_amd/lib/$1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "fused_adam or large_batch" -x -q --timeout 120 --timeout-method thread > gpurun_out/red/pytest.log 2>&1; rc=$?; tail -1 gpurun_out/red/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_bench_multi.sh 3 libceo_tt.so "$@"
