#!/bin/bash
# round-4 first GPU pass: the new parity tests (kinks, INTEGRATION stub, bench
# --gpus launch, cfg-4 eight ranks, data-parallel train_model), then the bench
set -o pipefail
TAG=${1:-r04a}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest -v --timeout 400 --timeout-method thread -m gpu \
  tests/test_gpu_kinks.py tests/test_integration_doc.py "tests/test_gpu_peer_exchange.py" tests/test_bench_launch.py \
  "tests/test_gpu_training.py::test_train_model_data_parallel_two_ranks_one_gpu" tests/test_gpu_cfg4.py \
  > $OUT/tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR|passed|failed" $OUT/tests.log | tail -40
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench.json'));print('value',d['value'],'ms',d['ms_per_step']);print(d['kernel_us']);print('roof',d['roofline']['achieved'],d['roofline']['frac']);c=d['cosine_roofline'];print('cos',c['achieved'],c['frac'],'stream',c['stream_peak_measured'],c['torch_copy_gbs'],c['frac_of_measured_stream'])"
