#!/bin/bash
# tests + bench (no cpu baseline) + rocprofv3 kernel stats of the same bench; usage: bash tools/gpu_prof.sh <tag>
set -o pipefail
TAG=${1:-p}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x > $OUT/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { rc=$?; echo bench failed; tail $OUT/bench.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print(d['kernel_us']);print('roof',d['roofline']['achieved'],d['roofline']['frac'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/prof.log 2>&1 || { rc=$?; echo rocprof failed; tail $OUT/prof.log; exit $rc; }
python - <<PY
import csv,glob
f=glob.glob("$OUT/prof/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "tt::" in r["Name"]: print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1000,2))
PY
