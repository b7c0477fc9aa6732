# A/B of the cfg-5 contrastive leg (tools/nce_probe.py) over library builds, interleaved
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/nab
A=$1; B=$2; R=${3:-2}
for i in $(seq 1 $R); do
  for L in $A $B; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python tools/nce_probe.py ${NCE_B:-16384 100000} > gpurun_out/nab/$L.$i.txt 2>&1 || { echo "$L failed"; tail -5 gpurun_out/nab/$L.$i.txt; exit 1; }
    echo "== $L"; grep -v amdgpu.ids gpurun_out/nab/$L.$i.txt | tail -6
  done
done
