#!/bin/bash
# A/B of library builds: parity subset on the default library, then an
# interleaved bench of the given builds.
# usage: bash tools/gpu_ab.sh TAG ROUNDS "pytest selection" lib1.so[@bench args] lib2.so ...
set -o pipefail
TAG=$1; R=$2; SEL=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
if [ -n "$SEL" ]; then
  timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu $SEL > $OUT/tests.log 2>&1; rc=$?
  tail -3 $OUT/tests.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $OUT/tests.log | head -20; exit $rc; }
fi
for i in $(seq 1 $R); do
  for SPEC in "$@"; do
    L=${SPEC%%@*}; X=""; [ "$SPEC" != "$L" ] && X=${SPEC#*@}; X=${X//,/ }; T=$(echo "$SPEC" | tr '@ ,' '___')
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-contrastive --no-side-config --steps 400 $X > $OUT/$T.$i.json 2> $OUT/$T.$i.err || { echo "$SPEC failed"; tail -5 $OUT/$T.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$OUT/$T.$i.json'));k=d['kernel_us'];print('$SPEC', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
  done
done
