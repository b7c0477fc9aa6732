#!/bin/bash
# after the make_red fix: the deferred-step diagnostic, the deferral tests,
# then the round-final evidence (suite, smoke, bench, rocprof, PMC)
set -o pipefail
T=${1:-r04d}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 240 python -u tools/diag_defer.py > $D/diag.log 2>&1 || { tail -20 $D/diag.log; exit 1; }
tail -3 $D/diag.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -q -x --timeout 180 --timeout-method thread > $D/defer.log 2>&1 || { tail -30 $D/defer.log; exit 1; }
tail -1 $D/defer.log
bash tools/gpu_final.sh $T
