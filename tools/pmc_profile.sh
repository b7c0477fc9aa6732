#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter set) over a short bench.
# usage: bash tools/pmc_profile.sh <tag> [bench args]
#        PMC_CMD="tools/nce_probe.py 32768" PMC_SETS=3 bash tools/pmc_profile.sh <tag>   (another python program, first N sets)
set -o pipefail
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
BENCH=${PMC_CMD:-"bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --no-side-config --no-contrastive --no-train-entry $@"}
i=0
for SET in \
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM" \
  "FETCH_SIZE" "WRITE_SIZE" ; do
  i=$((i+1))
  [ -n "$PMC_SETS" ] && [ $i -gt $PMC_SETS ] && break
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || { rc=$?; echo "pass $i ($SET) failed rc=$rc"; tail -5 $OUT/p$i.log; exit $rc; }
done
ls -R $OUT | head -40
