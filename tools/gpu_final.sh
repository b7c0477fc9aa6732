# round-final evidence: GPU suite, smoke, the driver's bench command (K=20,
# W=5) and the default bench, rocprofv3 kernel stats (csv) of the bench,
# PMC HBM-traffic passes -> profiles
set -o pipefail
export TMPDIR=/tmp; T=${1:-r03final}; D=gpurun_out/$T; mkdir -p $D
timeout -k 10 700 python -u -m pytest tests -m gpu -q -x --timeout 180 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { tail -20 $D/smoke.log; exit 1; }
tail -1 $D/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench_k20.json 2> $D/bench_k20.err || { tail -20 $D/bench_k20.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench_k20.json'));print('K20', d['ms_per_step'], round(d['value']/1e6,1), d['roofline']['frac'])"
timeout -k 10 300 python bench.py > $D/bench.json 2> $D/bench.err || { tail -20 $D/bench.err; exit 1; }
python -c "import json;d=json.load(open('$D/bench.json'));print('K400', d['ms_per_step'], round(d['value']/1e6,1), d['kernel_us'], d['roofline']['frac'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-contrastive --no-train-entry > $D/prof.log 2>&1 || { rc=$?; tail -20 $D/prof.log; exit $rc; }
find $D/prof -name "*kernel_stats.csv"
bash tools/pmc_profile.sh $T/pmc > $D/pmc.log 2>&1 || { tail -20 $D/pmc.log; exit 1; }
python tools/pmc_traffic.py $D/pmc $D/pmc_traffic.json && echo pmc ok
# roctx ranges: the step / exchange entry points and bench's timed region in a marker trace
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d $D/markers -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $D/markers.log 2>&1 || { rc=$?; tail -20 $D/markers.log; exit $rc; }
find $D/markers -name "*.csv" | head
