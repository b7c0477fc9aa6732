# interleaved bench rounds under different environment settings:
#   bash tools/gpu_env_ab.sh ROUNDS "ENV1" "ENV2" ...   (ENV "-" = unchanged)
#   STEPS / WARMUP / BENCH_ARGS override the bench arguments
set -o pipefail
export TMPDIR=/tmp; mkdir -p gpurun_out/envab
R=$1; shift
for i in $(seq 1 $R); do
  j=0
  for E in "$@"; do
    j=$((j+1))
    if [ "$E" = "-" ]; then E=""; fi
    B=bench.py; EE=""
    for tok in $E; do
      case "$tok" in BENCH=*) B="${tok#BENCH=}";; *) EE="$EE $tok";; esac
    done
    E="$EE"
    env $E timeout -k 10 200 python $B ${BENCH_ARGS:---no-cpu-baseline --no-contrastive --no-side-config --no-train-entry} --steps ${STEPS:-400} --warmup ${WARMUP:-20} > gpurun_out/envab/$j.$i.json 2> gpurun_out/envab/$j.$i.err || { echo "$E failed"; tail -5 gpurun_out/envab/$j.$i.err; exit 1; }
    TAG="$E $B" F=gpurun_out/envab/$j.$i.json python - <<'PY'
import json, os
d = json.load(open(os.environ["F"]))
k = d.get("kernel_us", {})
print("[" + os.environ["TAG"] + "]", d["ms_per_step"], round(d["value"] / 1e6, 1), {a[2:]: round(b, 2) for a, b in k.items()})
PY
  done
done
