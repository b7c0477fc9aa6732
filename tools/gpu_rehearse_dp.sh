# N>1 rehearsal on a one-GPU box: 2 ranks on GPU 0 over gloo (RCCL refuses two
# ranks on one device), full bench incl. the sharded contrastive leg.
set -o pipefail
OUT=gpurun_out/dp2; mkdir -p $OUT; export TMPDIR=/tmp
CEO_BENCH_SHARE_GPU=1 CEO_BENCH_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node ${NP:-2} \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus ${NP:-2} --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; tail -5 $OUT/bench.err; cat $OUT/bench.json; exit $rc
