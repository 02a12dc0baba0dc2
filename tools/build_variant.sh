# Build libspe.so of git revision $1 into $2 (same-box A/B: SPE_LIB=$2/libspe.so python bench.py ...)
set -e
REV=$1; OUT=$2
mkdir -p $OUT/csrc $OUT/include
for f in spe.hip spe_graph_prep.cpp spe_multi.cpp spe_internal.h; do
  git show $REV:shadow_amd/csrc/$f > $OUT/csrc/$f 2>/dev/null || true
done
git show $REV:include/spe.h > $OUT/include/spe.h
sed -i 's|#include "../../include/spe.h"|#include "../include/spe.h"|' $OUT/csrc/spe_internal.h
SRCS="$OUT/csrc/spe.hip $OUT/csrc/spe_graph_prep.cpp"
[ -s $OUT/csrc/spe_multi.cpp ] && SRCS="$SRCS $OUT/csrc/spe_multi.cpp"
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -shared -o $OUT/libspe.so $SRCS -ldl -lpthread
echo built $OUT/libspe.so
