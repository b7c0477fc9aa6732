# flakiness check: the full GPU suite twice more (fresh processes) and the graph-replay loop
set -o pipefail
export TMPDIR=/tmp; D=gpurun_out/flaky; mkdir -p $D
for v in 1 2; do
  timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread -p no:randomly > $D/pytest_$v.log 2>&1; rc=$?
  echo "suite $v rc=$rc: $(tail -1 $D/pytest_$v.log)"; grep FAILED $D/pytest_$v.log | head -5
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 300 python -u tools/gpu_loop_graph.py $PWD 6 > $D/loop.log 2>&1; echo "loop rc=$?"; tail -2 $D/loop.log
