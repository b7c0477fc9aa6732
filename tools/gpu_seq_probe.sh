set -o pipefail
for i in 1 2; do
for v in 0 1; do
  if [ $v = 1 ]; then export CEO_BENCH_SEQ_ROWS=1; else unset CEO_BENCH_SEQ_ROWS; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --steps 400 > gpurun_out/seq$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/seq$v.json'));print('seq=$v', d['ms_per_step'], d['kernel_us'])"
done; done
