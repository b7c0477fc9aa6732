set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/r05c; mkdir -p $D
for W in 2 4 8; do
  for L in libceo_tt_r04.so libceo_tt.so; do
    CEO_TT_LIB=ceo-recommender_amd/lib/$L timeout -k 10 200 python tools/ar_timing.py $W 200 >> $D/ar.txt 2>> $D/ar.err || { echo "ar $W $L failed"; tail -20 $D/ar.err; exit 1; }
  done
done
cat $D/ar.txt
