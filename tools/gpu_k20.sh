# the driver's bench shape (K=20, W=5): graph chunk variants, interleaved rounds
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/k20b; mkdir -p $D
A="--gpus 1 --no-extras --no-cpu-baseline --no-contrastive --no-side-config"
for v in 1 2 3 4; do
  for c in 20 10 5 4; do
    CEO_BENCH_CHUNK_MAX=$c timeout -k 10 120 python bench.py $A --steps 20 --warmup 5 > $D/k20_c${c}_$v.json 2>>$D/err.log || exit 1
  done
  python -c "
import json
print('round $v K20 chunk 20/10/5/4', [json.load(open('$D/k20_c%s_$v.json'%c))['ms_per_step'] for c in (20,10,5,4)])"
done
