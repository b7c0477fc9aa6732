# full GPU suite, interleaved bench A/B of library builds, then the default bench.py once
# usage: bash tools/gpu_ab_bench.sh <tag> <rounds> lib1.so lib2.so ...
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/$1; mkdir -p $D; shift
R=$1; shift
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -40 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
bash tools/gpu_bench_multi.sh $R "$@" || exit 1
timeout -k 10 400 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench.json'));print('bench', d['ms_per_step'], d['value']/1e6, d['roofline']['frac'], d.get('extras_error'), d['contrastive']['ms_per_step'], d['cpu_baseline']['value'])"
