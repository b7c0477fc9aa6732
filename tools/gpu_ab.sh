# A/B a test selection over library builds with a NaN-poisoned module workspace
# usage: bash tools/gpu_ab.sh "<pytest -k expr>" lib1 [lib2 ...]
export TMPDIR=/tmp; mkdir -p gpurun_out/ab
K="$1"; shift
for L in "$@"; do
  CEO_TT_POISON_WS=1 CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -k "$K" > gpurun_out/ab/$L.log 2>&1; echo "$L rc=$?"; grep -E "^(FAILED|E .*assert)" gpurun_out/ab/$L.log | head -12; tail -1 gpurun_out/ab/$L.log
done
