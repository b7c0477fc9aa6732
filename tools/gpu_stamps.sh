export TMPDIR=/tmp; mkdir -p gpurun_out/st
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg3 > gpurun_out/st/stamps.txt 2>&1; grep -v amdgpu.ids gpurun_out/st/stamps.txt
