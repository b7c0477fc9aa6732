# A/B bench of library builds on one box, interleaved: usage bash tools/gpu_bench_ab.sh libA.so libB.so [rounds]
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/bab
A=$1; B=$2; R=${3:-3}
for i in $(seq 1 $R); do
  for L in $A $B; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --steps 400 > gpurun_out/bab/$L.$i.json 2> gpurun_out/bab/$L.$i.err || { echo "$L failed"; tail -5 gpurun_out/bab/$L.$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/bab/$L.$i.json'));print('$L', d['ms_per_step'], round(d['value']/1e6,1), d['kernel_us'], d['cosine_roofline']['avg_us'])"
  done
done
