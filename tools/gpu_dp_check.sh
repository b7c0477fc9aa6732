set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/dp1
timeout -k 10 300 python bench.py --dp --steps 200 --warmup 10 --no-cpu-baseline --no-contrastive > gpurun_out/dp1/bench.json 2> gpurun_out/dp1/bench.err || { echo dp1 failed; tail gpurun_out/dp1/bench.err; exit 1; }
cat gpurun_out/dp1/bench.json
CEO_TT_PEER_AR=1 bash tools/gpu_rehearse_dp.sh
