# interleaved A/B of the plain step vs the deferred late half (bench --defer), cfg 3, K = 400
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/dab
for i in 1 2 3; do
  for a in plain defer; do
    arg=""; [ $a = defer ] && arg="--defer"
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --no-side-config --no-train-entry --steps 400 --warmup 20 $arg > gpurun_out/dab/$a.$i.json 2> gpurun_out/dab/$a.$i.err || { tail -5 gpurun_out/dab/$a.$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/dab/$a.$i.json'));k=d['kernel_us'];print('$a', d['ms_per_step'], round(d['value']/1e6,1), {x[2:]: round(y,2) for x,y in k.items()})"
  done
done
