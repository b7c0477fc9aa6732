# stamps of the plain stamps build and of a diagnostic variant, one box
export TMPDIR=/tmp; mkdir -p gpurun_out/st
for L in ${LIBS:-libceo_tt_stamps.so libceo_tt_stamps_diag.so}; do
  echo "== $L"
  CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python tools/stamps.py cfg3 > gpurun_out/st/$L.txt 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/st/$L.txt | grep -v "^$"
done
