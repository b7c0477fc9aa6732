mkdir -p gpurun_out/s3; export TMPDIR=/tmp
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -q -x > gpurun_out/s3/pt.log 2>&1 || { tail gpurun_out/s3/pt.log; exit 1; }
tail -1 gpurun_out/s3/pt.log
STAMPS_ROWS=10000000 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/s3/p -o run --output-format csv -- python3 tools/stamps_prod.py > gpurun_out/s3/p.log 2>&1 || { tail gpurun_out/s3/p.log; exit 1; }
python - <<PY
import csv,glob
f=glob.glob("gpurun_out/s3/p/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "tt::" in r["Name"]: print(r["Name"][:50], r["Calls"], round(float(r["AverageNs"])/1000,2))
PY
