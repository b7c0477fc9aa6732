# stamps of experiment libraries: bash tools/gpu_stamps_x.sh lib1 lib2 ...
export TMPDIR=/tmp; mkdir -p gpurun_out/stx
for L in "$@"; do
  echo "== $L"
  CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python tools/stamps.py cfg3 > gpurun_out/stx/$L.txt 2>&1 || { echo "failed $L"; tail -5 gpurun_out/stx/$L.txt; exit 1; }
  grep -A9 "^k_top" gpurun_out/stx/$L.txt | head -10
done
