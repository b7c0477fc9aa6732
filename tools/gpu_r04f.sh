#!/bin/bash
# cosine grid / stream copy change: the cosine + ABI tests, the bench extras
# (cosine_roofline with the new stream ceiling); cfg-2 per-phase stamps
set -o pipefail
T=${1:-r04f}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "cosine or abi" -q -x --timeout 180 --timeout-method thread > $D/cos.log 2>&1 || { tail -30 $D/cos.log; exit 1; }
tail -1 $D/cos.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-contrastive > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench.json'));print(d['ms_per_step'], d['value']/1e6, d['cosine_roofline'], d['other_configs'])"
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg2 > $D/stamps_cfg2.txt 2>&1 || { tail $D/stamps_cfg2.txt; exit 1; }
grep -v amdgpu.ids $D/stamps_cfg2.txt
