# contrastive GPU parity tests, then an interleaved A/B of the cfg-5 leg: bash tools/gpu_nce_check.sh base.so new.so
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/nab
timeout -k 10 300 python -u -m pytest tests -m gpu -k "contrastive or nce or rank or triplet or semi" -x -q --timeout 120 --timeout-method thread > gpurun_out/nab/pytest.log 2>&1; rc=$?; tail -2 gpurun_out/nab/pytest.log; [ $rc -eq 0 ] || exit $rc
NCE_B=100000 bash tools/gpu_nce_ab.sh $1 $2 2
