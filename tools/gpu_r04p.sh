#!/bin/bash
# probe: k_reduce_adam with the Adam state (p, m, v) loaded after the slab
# sums (TT_RED_PMV_LATE) -- per-block stamps and an interleaved A/B
set -o pipefail
T=${1:-r04p}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 env CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_pmv.so python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 180 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
STAMPS_BLOCKS=1 CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_pmvst.so timeout -k 10 200 python tools/stamps.py cfg3 > $D/stamps_cfg3.txt 2>&1 || { tail -5 $D/stamps_cfg3.txt; exit 1; }
B="--no-cpu-baseline --no-contrastive --no-side-config"
for i in 1 2 3; do
  for L in libceo_tt.so libceo_tt_pmv.so; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py $B --steps 400 > $D/$L.$i.json 2> $D/$L.$i.err || { tail -5 $D/$L.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$L.$i.json'));k=d.get('kernel_us',{});print('$L', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
grep "blocks " $D/stamps_cfg3.txt | awk 'NR%3==1'
