#!/bin/bash
# k_reduce_adam element-space order: HEAD (tower order) vs heaviest first vs
# heaviest first with tower 1 ahead; full GPU suite on the heaviest-first build
set -o pipefail
T=${1:-r04o}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
B="--no-cpu-baseline --no-contrastive --no-side-config"
for i in 1 2 3; do
  for L in libceo_tt_base.so libceo_tt.so libceo_tt_t1.so; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py $B --steps 400 > $D/$L.$i.json 2> $D/$L.$i.err || { tail -5 $D/$L.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$L.$i.json'));k=d.get('kernel_us',{});print('$L', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
