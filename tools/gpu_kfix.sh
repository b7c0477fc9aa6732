# fixed per-run overhead of the timed region: single-graph runs at K = 1..40
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/kfix; mkdir -p $D
A="--gpus 1 --no-extras --no-cpu-baseline --no-contrastive --no-side-config"
for v in 1 2; do
for k in 1 2 5 10 20 40; do
  CEO_BENCH_CHUNK_MAX=$k timeout -k 10 120 python bench.py $A --steps $k --warmup 5 > $D/k${k}_$v.json 2>>$D/err.log || exit 1
done
python -c "
import json
for k in (1,2,5,10,20,40):
    d=json.load(open('$D/k%d_$v.json'%k)); print(k, round(d['ms_per_step']*k*1000,1), 'us total', d['ms_per_step'])"
done
