# timing-only upper bound: the step with the late half of the reduction (W4 / BN1 / W8 / logit_scale) dropped
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/nolate; mkdir -p $D
A="--gpus 1 --no-cpu-baseline --no-contrastive --no-side-config"
for v in 1 2 3; do
  timeout -k 10 120 python bench.py $A > $D/base_$v.json 2>>$D/err.log || exit 1
  CEO_TT_LIB=$PWD/ceo-recommender_amd/lib/libceo_tt_probe_nolate.so timeout -k 10 120 python bench.py $A > $D/probe_$v.json 2>>$D/err.log || exit 1
  python -c "
import json
a=json.load(open('$D/base_$v.json'));b=json.load(open('$D/probe_$v.json'))
print('round $v base', a['ms_per_step'], a['kernel_us']['k_reduce_adam'], ' no-late', b['ms_per_step'], b['kernel_us']['k_reduce_adam'])"
done
