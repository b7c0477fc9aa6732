#!/bin/bash
# bench single / data-parallel (world 1, RCCL) graph and eager; usage: bash tools/gpu_dp_probe.sh <tag>
set -o pipefail
TAG=${1:-dp}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/single.json 2> $OUT/single.err || { rc=$?; echo single failed; tail $OUT/single.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/single.json'));print('single',d['value'],d['ms_per_step'],d['kernel_us'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --dp > $OUT/dp_graph.json 2> $OUT/dp_graph.err || { rc=$?; echo dp graph failed; tail $OUT/dp_graph.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/dp_graph.json'));print('dp graph',d['value'],d['ms_per_step'],d['mean_loss'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --dp --no-graph > $OUT/dp_eager.json 2> $OUT/dp_eager.err || { rc=$?; echo dp eager failed; tail $OUT/dp_eager.err; exit $rc; }
python -c "import json;d=json.load(open('$OUT/dp_eager.json'));print('dp eager',d['value'],d['ms_per_step'],d['mean_loss'])"
