# build lib/libceo_tt_<tag>.so from the working tree with extra defines, for A/B runs:
#   bash tools/build_variant.sh TAG -DTT_X=0 ...
TAG=$1; shift
cd "$(dirname "$0")/../ceo-recommender_amd/csrc" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -Wno-unused-result "$@" tt_abi.hip -o ../lib/libceo_tt_$TAG.so -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib && echo built libceo_tt_$TAG.so
