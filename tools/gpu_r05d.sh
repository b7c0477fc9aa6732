# round 5: K = 20 fixed cost (chunk lists, spin sync) + k_l4_fwd shift A/B
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/r05d; mkdir -p $D
timeout -k 10 300 python tools/kfix_probe.py 20 25 > $D/kfix.txt 2>$D/kfix.err || { tail $D/kfix.err; exit 1; }
CEO_PROBE_SPIN=1 timeout -k 10 300 python tools/kfix_probe.py 20 25 > $D/kfix_spin.txt 2>$D/kfix_spin.err || { tail $D/kfix_spin.err; exit 1; }
cat $D/kfix.txt $D/kfix_spin.txt
bash tools/gpu_bench_multi.sh 3 libceo_tt.so libceo_tt_l4sh.so libceo_tt_pf.so
