set -o pipefail
mkdir -p gpurun_out/q
timeout -k 10 300 python -u -m pytest tests/test_gpu_contrastive.py -x -v --timeout 120 --timeout-method thread -k "semi_hard or info_nce_golden" > gpurun_out/q/t.log 2>&1; rc=$?; tail -25 gpurun_out/q/t.log; exit $rc
