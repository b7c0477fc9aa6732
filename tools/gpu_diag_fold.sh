# stress: first-step gradient vs oracle at B = 16384, atomic mode, 8 reps per build
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/${DD:-diag4}; mkdir -p $D
export DIAG_REPS=8 DIAG_ATOMIC_ONLY=1
for v in ${VARIANTS:-head l_awall l_l4wait l_safeatom}; do
  if [ $v = head ]; then L=""; else L=$PWD/ceo-recommender_amd/lib/bisect/$v.so; fi
  CEO_TT_LIB=$L timeout -k 10 200 python -u tools/diag_fold16k.py 16384 > $D/$v.log 2>&1 || { tail -20 $D/$v.log; exit 1; }
  echo "== $v: $(grep -c 'ceo_tower.5.bias .*FAIL\|firm_tower.5.bias .*FAIL' $D/$v.log) failing reps of $(grep -c 'rep=' $D/$v.log)"; grep "worst ch.*diff [0-9.-]*e-0[0-4]\|FAIL" $D/$v.log | grep "worst\|5.bias" | head -4
done
