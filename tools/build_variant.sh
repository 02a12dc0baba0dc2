# Build an experimental libspe.so with extra compiler flags into build_ab/<name>/
# (A/B runs select it with SPE_LIB; never the shipped library).
#   bash tools/build_variant.sh <name> [-DFLAG=...]...
set -e
N=$1; shift
mkdir -p build_ab/$N
C=shadow_amd/csrc
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -Wall -Wno-unused-function "$@" \
  -shared -o build_ab/$N/libspe.so $C/spe.hip $C/spe_graph_prep.cpp $C/spe_multi.cpp -ldl -lpthread
echo "built build_ab/$N/libspe.so ($*)"
