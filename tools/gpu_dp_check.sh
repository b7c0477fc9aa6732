#!/bin/bash
# Data-parallel exchange check on the one-GPU box: the peer-exchange tests
# (2 / 4 ranks sharing the GPU, the in-reduction exchange, timeouts), then
# bench at world size 1 single vs --dp (the N > 1 step's cost with nothing to
# exchange).  Each GPU step under its own limit; the first failure ends it.
set -o pipefail
OUT=gpurun_out/${1:-dp}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_peer_exchange.py -x -v --timeout 180 --timeout-method thread > $OUT/pytest_peer.log 2>&1
rc=$?; echo "pytest_peer rc=$rc"; tail -15 $OUT/pytest_peer.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 400 --warmup 50 --no-extras --no-cpu-baseline --no-side-config --no-contrastive > $OUT/bench_single_$i.json 2> $OUT/bench_single_$i.err || { echo "bench single failed"; tail $OUT/bench_single_$i.err; exit 1; }
  timeout -k 10 300 python bench.py --dp --steps 400 --warmup 50 --no-extras --no-cpu-baseline --no-side-config --no-contrastive > $OUT/bench_dp_$i.json 2> $OUT/bench_dp_$i.err || { echo "bench dp failed"; tail $OUT/bench_dp_$i.err; exit 1; }
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/*/bench_*_[12].json")):
    try:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(f, d["ms_per_step"], d["config"]["parallelism"], d["config"]["grad_exchange"])
    except Exception as e:
        print(f, "unreadable", e)
PY
