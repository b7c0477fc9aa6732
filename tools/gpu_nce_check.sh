# contrastive GPU parity tests, then an interleaved A/B of the cfg-5 kernels against a baseline build
# (bash tools/build_base.sh <rev> base first: ceo-recommender_amd/lib/libceo_tt_base.so)
set -o pipefail
mkdir -p gpurun_out/nab
timeout -k 10 400 python -u -m pytest tests -m gpu -k "contrastive or nce or rank or triplet or semi" -x -q --timeout 200 --timeout-method thread > gpurun_out/nab/pytest.log 2>&1 || { tail -20 gpurun_out/nab/pytest.log; exit 1; }
tail -1 gpurun_out/nab/pytest.log
bash tools/gpu_nce_ab.sh 2 libceo_tt_base.so libceo_tt.so
