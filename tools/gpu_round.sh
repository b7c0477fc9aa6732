#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace
# summary of the same bench command, and (with PMC=1) the HBM-traffic passes.
# Every GPU step has its own time limit; the first failure ends the script.
# usage: [PMC=1] bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest_gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { rc=$?; echo "smoke failed rc=$rc"; tail $OUT/smoke.log; exit $rc; }
tail -1 $OUT/smoke.log
timeout -k 10 500 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { rc=$?; echo "bench failed rc=$rc"; tail -20 $OUT/bench.err; exit $rc; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline "$@" > $OUT/prof.log 2>&1 || { rc=$?; echo "rocprof failed rc=$rc"; tail -20 $OUT/prof.log; exit $rc; }
find $OUT/prof -name "*kernel_stats.csv"
if [ "${PMC:-0}" = "1" ]; then
  bash tools/pmc_profile.sh $TAG/pmc "$@" || exit $?
  python tools/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic.json
fi
