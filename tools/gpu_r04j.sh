#!/bin/bash
# 32-row tower kernels below the folded path: GPU suite, then interleaved
# cfg-2 A/B: every kernel on 64-row tiles, k_top_pair alone on 32, all on 32
set -o pipefail
T=${1:-r04j}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
B="--no-cpu-baseline --no-contrastive --no-side-config"
for i in 1 2 3; do
  for L in libceo_tt_all64.so libceo_tt_pair32.so libceo_tt.so; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py $B --config cfg2 --steps 400 > $D/$L.cfg2.$i.json 2> $D/$L.cfg2.$i.err || { tail -5 $D/$L.cfg2.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$L.cfg2.$i.json'));k=d.get('kernel_us',{});print('$L cfg2', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
timeout -k 10 200 python bench.py $B --no-extras --steps 400 > $D/cfg3.json 2> $D/cfg3.err || { tail -5 $D/cfg3.err; exit 1; }
python -c "import json;d=json.load(open('$D/cfg3.json'));print('cfg3', d['ms_per_step'], round(d['value']/1e6,1))"
