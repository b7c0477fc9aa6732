# interleaved bench of several library builds on one box: bash tools/gpu_bench_multi.sh rounds lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/bm
R=$1; shift
for i in $(seq 1 $R); do
  for L in "$@"; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --steps 400 > gpurun_out/bm/$L.$i.json 2> gpurun_out/bm/$L.$i.err || { echo "$L failed"; tail -5 gpurun_out/bm/$L.$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bm/$L.$i.json'));k=d['kernel_us'];print('$L', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
