# quick GPU check: the named pytest files (default: every gpu test), one process, each test bounded
set -o pipefail
mkdir -p gpurun_out/q
FILES=${@:-tests}
timeout -k 10 500 python -u -m pytest $FILES -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/q/t.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/q/t.log | tail -60; [ $rc -eq 0 ] || tail -60 gpurun_out/q/t.log; exit $rc
