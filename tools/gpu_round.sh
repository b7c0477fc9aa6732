#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel-trace summary.
# usage: bash tools/gpu_round.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-dev}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q > $OUT/pytest_gpu.log 2>&1
echo "pytest_gpu rc=$?" | tee -a $OUT/status.log
tail -3 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python bench.py "$@" > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed"; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --no-cpu-baseline --no-graph > $OUT/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -3
