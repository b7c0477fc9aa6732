set -o pipefail
bash tools/gpu_bench_multi.sh 2 libceo_tt_r05.so && bash tools/gpu_stamps.sh
