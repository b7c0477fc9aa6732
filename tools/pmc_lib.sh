set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmcf2; mkdir -p $OUT
BENCH="bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-graph --no-side-config --no-contrastive --no-extras"
i=0
for SET in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_MFMA" "FETCH_SIZE"; do
  i=$((i+1))
  CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_f2.so timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_summary.py $OUT
