mkdir -p gpurun_out/c4; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4/p -o run --output-format csv -- python3 tools/nce_probe.py 100000 > gpurun_out/c4/p.log 2>&1 || { tail gpurun_out/c4/p.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob("gpurun_out/c4/p/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "nce" in r["Name"]: print(r["Name"][:60], r["Calls"], round(float(r["AverageNs"])/1e6,3), "ms")
PY
for SET in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" "SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS" "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/c4/pmc$i -o run -- python3 tools/nce_probe.py 16384 > gpurun_out/c4/pmc$i.log 2>&1 || { tail -5 gpurun_out/c4/pmc$i.log; exit 1; }
done
python tools/pmc_summary.py gpurun_out/c4 nce
