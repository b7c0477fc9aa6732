# the driver's bench shape (K=20, W=5) vs K=400: graph chunking variants, interleaved
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/k20; mkdir -p $D
A="--gpus 1 --no-extras --no-cpu-baseline --no-contrastive --no-side-config"
for v in 1 2 3; do
  for c in 16 20 10; do
    CEO_BENCH_CHUNK_MAX=$c timeout -k 10 120 python bench.py $A --steps 20 --warmup 5 > $D/k20_c${c}_$v.json 2>>$D/err.log || exit 1
  done
  timeout -k 10 120 python bench.py $A --steps 400 --warmup 20 > $D/k400_$v.json 2>>$D/err.log || exit 1
  python -c "
import json
r=[json.load(open('$D/k20_c%s_$v.json'%c))['ms_per_step'] for c in (16,20,10)]
print('round $v K20 chunk16/20/10', r, 'K400', json.load(open('$D/k400_$v.json'))['ms_per_step'])"
done
