# full GPU suite on the in-tree build, then an interleaved bench A/B of library builds
# usage: bash tools/gpu_ab_full.sh <tag> <rounds> lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/$1; mkdir -p $D; shift
R=$1; shift
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
bash tools/gpu_bench_multi.sh $R "$@"
