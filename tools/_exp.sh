mkdir -p gpurun_out/dp2; export TMPDIR=/tmp
CEO_BENCH_SHARE_GPU=1 CEO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dp2/out.json 2> gpurun_out/dp2/err.log; rc=$?
echo "rc=$rc"; tail -c 2500 gpurun_out/dp2/out.json; grep -iE "error|Traceback" -A3 gpurun_out/dp2/err.log | head -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --dp --no-graph --no-cpu-baseline --no-extras > gpurun_out/dp2/dp_eager.json 2>gpurun_out/dp2/dp_eager.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/dp2/dp_eager.json'));print('dp eager world1', d['value'], d['ms_per_step'])"
