# Same-box A/B of relaxation variants on whole C3 / C4 tables, alternating
# $REPS times.  A variant is lib:relax:rows:occ -- lib "tree" = the in-tree
# libspe.so, else build_ab/<lib>/libspe.so (SPE_LIB); relax = SPE_RELAX (1
# k_relax_m, 2 k_relax_s), rows / occ = SPE_INFL / SPE_OCC (0 = default).
set -e
O=gpurun_out/${TAG:-relax_ab}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for V in ${VARIANTS:-tree:1:0:0 tree:2:0:0}; do
    IFS=: read -r LIB RX RW OC <<< "$V"
    for C in ${CONFIGS:-c3 c4}; do
      F=$O/b_${C}_${LIB}_${RX}_${RW}_${OC}_$rep.log
      if [ "$LIB" = tree ]; then unset SPE_LIB; else export SPE_LIB=$PWD/build_ab/$LIB/libspe.so; fi
      SPE_RELAX=$RX SPE_INFL=$RW SPE_OCC=$OC timeout -k 10 240 python -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-side $EXTRA > $F 2>&1 || { tail -20 $F; exit 1; }
      python - $F "$C $V rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r=l["roofline"]
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "avg_us", r["launch_avg_us"], "frac", r["frac"], "rounds", l["relax_rounds_per_step"], "relax_ms", l["kernel_ms"]["relax"])
PY
    done
  done
done
unset SPE_LIB
