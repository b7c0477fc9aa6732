# A/B of train()'s rate (bench's train_entry leg) under CEO_TT_STAGE_ORDER=1 / 0 (the staging knob measured in round 5 was removed)
set -o pipefail
mkdir -p gpurun_out/tab
timeout -k 10 300 python -u -m pytest tests/test_gpu_training.py -x -q --timeout 200 --timeout-method thread > gpurun_out/tab/pytest.log 2>&1 || { tail -20 gpurun_out/tab/pytest.log; exit 1; }
tail -1 gpurun_out/tab/pytest.log
for r in 1 2 3; do
  for st in 1 0; do
    CEO_TT_STAGE_ORDER=$st timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-contrastive --no-side-config > gpurun_out/tab/b_${r}_$st.json 2> gpurun_out/tab/b_${r}_$st.err || { tail -5 gpurun_out/tab/b_${r}_$st.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/tab/b_${r}_$st.json'));t=d['train_entry'];print('r$r stage=$st', t['us_per_step'], t['ms_per_epoch'], round(t['train_entry_pairs_per_s']/1e6,1), 'headline', d['ms_per_step'])"
  done
done
