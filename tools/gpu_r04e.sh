#!/bin/bash
# copy-variant probe (stream ceiling), then interleaved A/B of the deferred
# late half (--defer) against plain steps: K = 400 and the driver's K = 20
set -o pipefail
T=${1:-r04e}; D=gpurun_out/$T; mkdir -p $D; export TMPDIR=/tmp
timeout -k 10 120 python tools/copyprobe/copy_probe.py > $D/copy.txt 2>&1 || { tail $D/copy.txt; exit 1; }
cat $D/copy.txt
B="--no-cpu-baseline --no-contrastive --no-side-config"
for i in 1 2 3; do
  for m in plain defer; do
    a=""; [ $m = defer ] && a="--defer"
    timeout -k 10 200 python bench.py $B --steps 400 $a > $D/$m.$i.json 2> $D/$m.$i.err || { tail -5 $D/$m.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$m.$i.json'));k=d['kernel_us'];print('$m K400', d['ms_per_step'], round(d['value']/1e6,1), {a[2:]: round(b,2) for a,b in k.items()})"
    timeout -k 10 200 python bench.py $B --steps 20 --warmup 5 $a > $D/$m.k20.$i.json 2> $D/$m.k20.$i.err || { tail -5 $D/$m.k20.$i.err; exit 1; }
    python -c "import json;d=json.load(open('$D/$m.k20.$i.json'));print('$m K20', d['ms_per_step'], round(d['value']/1e6,1))"
  done
done
