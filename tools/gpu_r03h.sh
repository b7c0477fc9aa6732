# session check: full GPU suite, smoke, the driver's bench command (K=20,
# W=5), the default long bench, rocprofv3 kernel stats of the bench
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/${1:-r03h}; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
echo smoke ok
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_k20.json 2> $D/bench_k20.err || { tail -20 $D/bench_k20.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench_k20.json'));print('K20', d['ms_per_step'], d['value']/1e6, d['kernel_us'], d['roofline']['frac'])"
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench.json'));print('K400', d['ms_per_step'], d['value']/1e6, d['kernel_us'], d['roofline']['frac'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$D/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-contrastive --steps 400 > $GRAFT_REPO_ROOT/$D/prof_bench.json 2> $GRAFT_REPO_ROOT/$D/prof.err || { tail -20 $GRAFT_REPO_ROOT/$D/prof.err; exit 1; }
echo prof ok
