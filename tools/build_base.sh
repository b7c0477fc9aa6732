# build lib/libceo_tt_<tag>.so from the sources at git revision REV (default HEAD) for A/B runs
REV=${1:-HEAD}; TAG=${2:-base}
D=/tmp/tt_base_$TAG; rm -rf $D; mkdir -p $D/csrc $D/include
for f in $(git ls-files ceo-recommender_amd/csrc include); do mkdir -p $D/$(dirname ${f#ceo-recommender_amd/}); git show $REV:$f > $D/${f#ceo-recommender_amd/}; done
sed -i 's#../../include/#../include/#' $D/csrc/*.hip $D/csrc/*.h 2>/dev/null
(cd $D/csrc && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -munsafe-fp-atomics -Wno-unused-result tt_abi.hip -o /root/repo/ceo-recommender_amd/lib/libceo_tt_$TAG.so -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib) && echo built libceo_tt_$TAG.so
