set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/r05e; mkdir -p $D
CEO_PROBE_VARIANTS="10+10,4+4+4+4+4,5+5+5+5,2+2+2+2+2+2+2+2+2+2,1+1+1+1+1+1+1+1+1+1+1+1+1+1+1+1+1+1+1+1,2+4+4+4+6,3+3+3+3+4+4" timeout -k 10 400 python tools/kfix_probe.py 20 25 > $D/kfix.txt 2>$D/kfix.err || { tail $D/kfix.err; exit 1; }
cat $D/kfix.txt
