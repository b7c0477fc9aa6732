set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1; echo "pytest rc=$?"; tail -2 gpurun_out/final/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/final/smoke.log
timeout -k 10 300 python -u tools/gpu_loop_graph.py $PWD 6 > gpurun_out/final/loop.log 2>&1; echo "loop rc=$?"; tail -1 gpurun_out/final/loop.log
