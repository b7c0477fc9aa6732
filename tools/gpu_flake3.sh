#!/bin/bash
# the GPU suite three times in a row (numerical flakes of atomic-order
# tolerances); stops at once on anything but pass / test failure
D=gpurun_out/flake; mkdir -p $D
for i in 1 2 3; do
  timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $D/run$i.log 2>&1
  rc=$?; tail -1 $D/run$i.log; grep FAILED $D/run$i.log
  [ $rc -le 1 ] || { echo "rc=$rc: stop"; exit $rc; }
done
