# gather-locality probe: the cfg-3 bench with the permutation (default) and with in-order rows
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/seq
for i in 1 2; do
  for SEQ in "" 1; do
    CEO_BENCH_SEQ_ROWS=$SEQ timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --no-side-config > gpurun_out/seq/b$SEQ.$i.json 2> gpurun_out/seq/b$SEQ.$i.err || { echo failed; tail -5 gpurun_out/seq/b$SEQ.$i.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/seq/b$SEQ.$i.json'));k=d['kernel_us'];print('seq=$SEQ', d['ms_per_step'], {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
