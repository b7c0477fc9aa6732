#!/bin/bash
# parity of the current build (incl. the deferred late half), A/B bench vs
# earlier builds, stamps + PMC of the current build
set -o pipefail
TAG=${1:-r04c}; OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_ab.sh $TAG 2 "tests/test_gpu_defer.py tests/test_gpu_kinks.py tests/test_gpu_parity.py tests/test_gpu_deterministic.py tests/test_gpu_peer_exchange.py tests/test_gpu_training.py" libceo_tt_base.so@--no-defer libceo_tt_new.so@--no-defer libceo_tt.so@--no-defer libceo_tt.so || exit 1
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg3 > $OUT/stamps.txt 2>&1 || { tail $OUT/stamps.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps.txt
CEO_TT_LIB=ceo-recommender_amd/lib/libceo_tt_stamps.so timeout -k 10 200 python tools/stamps.py cfg2 > $OUT/stamps_cfg2.txt 2>&1 || { tail $OUT/stamps_cfg2.txt; exit 1; }
grep -v amdgpu.ids $OUT/stamps_cfg2.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_cfg2 -o run -- python bench.py --config cfg2 --steps 200 --warmup 20 --no-extras --no-contrastive --no-side-config --no-cpu-baseline > $OUT/cfg2_prof.log 2>&1 || { tail $OUT/cfg2_prof.log; exit 1; }
find $OUT/prof_cfg2 -name '*kernel_stats.csv' -exec cut -d, -f1-8 {} \;
timeout -k 10 120 python tools/copyprobe/copy_probe.py > $OUT/copy.txt 2>&1 || { tail $OUT/copy.txt; exit 1; }
cat $OUT/copy.txt
bash tools/pmc_profile.sh $TAG/pmc > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
python tools/pmc_summary.py $OUT/pmc > $OUT/pmc_summary.txt 2>&1
python tools/pmc_traffic.py $OUT/pmc $OUT/pmc_traffic.json > $OUT/traffic.log 2>&1 && echo pmc ok
grep -E "k_(l0|l4|top|bwd|reduce)" $OUT/pmc_summary.txt | cut -c1-400
