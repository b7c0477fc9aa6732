#!/bin/bash
# parity tests + bench (no extras) + stamps; usage: bash tools/gpu_quick.sh <tag>
set -o pipefail
TAG=${1:-q}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print(d['kernel_us']);print('roof',d['roofline']['achieved'],d['roofline']['frac'],'cos',d['cosine_roofline']['frac'])"
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg3 > $OUT/stamps.txt 2>&1; grep -v amdgpu.ids $OUT/stamps.txt
