# Build libspe.so of the working tree with extra compiler flags into $1 (same-box A/B:
# SPE_LIB=$1/libspe.so python bench.py ...), e.g. tools/build_flags_variant.sh build_ab/win4 -DLDS_WIN_N=4
set -e
OUT=$1; shift
mkdir -p $OUT
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -shared "$@" \
  -o $OUT/libspe.so shadow_amd/csrc/spe.hip shadow_amd/csrc/spe_graph_prep.cpp shadow_amd/csrc/spe_multi.cpp -ldl -lpthread
echo built $OUT/libspe.so
