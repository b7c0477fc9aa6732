# full GPU suite + per-phase stamps of the cfg-3 step
set -o pipefail
export TMPDIR=/tmp; T=${1:-suite}; D=gpurun_out/$T; mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -30 $D/pytest_gpu.log; exit 1; }
tail -1 $D/pytest_gpu.log
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg3 > $D/stamps_cfg3.txt 2>&1 || { tail $D/stamps_cfg3.txt; exit 1; }
grep -v amdgpu.ids $D/stamps_cfg3.txt
