#!/bin/bash
# selected GPU tests, then (optionally) the default bench:
#   bash tools/gpu_sel.sh TAG "pytest selection" [bench args | nobench]
set -o pipefail
export TMPDIR=/tmp
T=${1:-sel}; SEL=${2:-tests -m gpu}; BARGS=${3:-}
D=gpurun_out/$T; mkdir -p $D
timeout -k 10 900 python -u -m pytest $SEL -x -v -s --timeout 600 --timeout-method thread > $D/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed|us \(|world [0-9]|rccl dp1" $D/pytest.log | tail -40
[ $rc -eq 0 ] || { tail -40 $D/pytest.log; exit $rc; }
[ "$BARGS" = "nobench" ] && exit 0
timeout -k 10 600 python bench.py $BARGS > $D/bench.json 2> $D/bench.err || { echo bench failed; tail -20 $D/bench.err; exit 1; }
python - <<PY
import json
d=json.load(open('$D/bench.json'))
print('value', d['value'], 'ms', d['ms_per_step'], 'roof', d.get('roofline',{}).get('frac'))
print('kernels', d.get('kernel_us'))
print('train_entry', d.get('train_entry'))
print('cos', (d.get('cosine_roofline') or {}).get('frac'), 'cfg2', (d.get('other_configs') or {}).get('cfg2'))
print('contrastive', {k: (d.get('contrastive') or {}).get(k) for k in ('ms_per_step','frac')})
print('extras_error', d.get('extras_error'))
PY
