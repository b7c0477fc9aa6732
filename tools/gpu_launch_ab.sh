# hipGraph replay vs one tt_train_steps call (C++ launch loop), K = 20 and 400, interleaved
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/lab; mkdir -p $D
A="--gpus 1 --no-extras --no-cpu-baseline --no-contrastive --no-side-config"
for v in 1 2 3; do
  for L in graph steps; do
    timeout -k 10 120 python bench.py $A --launch $L --steps 20 --warmup 5 > $D/k20_${L}_$v.json 2>>$D/err.log || { tail -5 $D/err.log; exit 1; }
    timeout -k 10 120 python bench.py $A --launch $L --steps 400 --warmup 20 > $D/k400_${L}_$v.json 2>>$D/err.log || { tail -5 $D/err.log; exit 1; }
  done
  python -c "
import json
r={L:[json.load(open('$D/k%d_%s_$v.json'%(k,L)))['ms_per_step'] for k in (20,400)] for L in ('graph','steps')}
print('round $v (K20, K400):', r)"
done
