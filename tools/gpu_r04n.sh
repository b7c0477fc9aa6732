#!/bin/bash
# k_reduce_adam element space heaviest range first; interleaved A/B vs HEAD
set -o pipefail
T=${1:-r04n}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kinks.py tests/test_gpu_deterministic.py tests/test_gpu_peer_exchange.py tests/test_gpu_defer.py tests/test_gpu_training.py -q -x --timeout 180 --timeout-method thread > $D/pytest.log 2>&1 || { tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
B="--no-cpu-baseline --no-contrastive --no-side-config"
for i in 1 2 3; do
  for L in libceo_tt_base.so libceo_tt.so; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py $B --steps 400 > $D/$L.$i.json 2> $D/$L.$i.err || { tail -5 $D/$L.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$L.$i.json'));k=d.get('kernel_us',{});print('$L', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
for c in cfg3; do
  STAMPS_BLOCKS=1 CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py $c > $D/stamps_$c.txt 2>&1 || { tail -5 $D/stamps_$c.txt; exit 1; }
done
tail -45 $D/stamps_cfg3.txt
