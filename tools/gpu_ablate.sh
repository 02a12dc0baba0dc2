# Upper bounds of k_relax components (diagnostic build, inexact rows): SPE_ABLATE bit 0 = no route
# records, bit 1 = no parent refreshes; alternating on one box.  Build the variant on the CPU first:
#   hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fno-fast-math -fPIC -std=c++17 -DSPE_DIAGNOSTICS -shared \
#     -o build_diag/libspe.so shadow_amd/csrc/spe.hip shadow_amd/csrc/spe_graph_prep.cpp shadow_amd/csrc/spe_multi.cpp -ldl -lpthread
set -e
O=gpurun_out/${TAG:-ablate}; mkdir -p $O
export SPE_LIB=$PWD/build_diag/libspe.so
for r in 1 2; do
  for C in c3 c4; do
    for A in 0 2 1; do
      LOG=$O/${C}_a${A}_$r.log
      SPE_ABLATE=$A timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$C ablate=$A run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'], d['relax_rounds_per_step'])"
    done
  done
done
