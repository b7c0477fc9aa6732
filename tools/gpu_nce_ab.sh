# interleaved A/B of the cfg-5 contrastive kernels: bash tools/gpu_nce_ab.sh R lib1.so lib2.so ...
# (each round runs tools/nce_probe.py at N = ${NCE_B:-100000} once per library)
set -o pipefail
R=$1; shift; mkdir -p gpurun_out/nab
for r in $(seq 1 $R); do
  for lib in "$@"; do
    echo -n "r$r $lib: "
    CEO_TT_LIB=ceo-recommender_amd/lib/$lib timeout -k 10 200 python tools/nce_probe.py ${NCE_B:-100000} 2> gpurun_out/nab/err_$lib.log || { tail -5 gpurun_out/nab/err_$lib.log; exit 1; }
  done
done
