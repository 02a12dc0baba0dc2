# Settle-bound A/B on C3 (round 6): per-round histograms from the SPE_RELAX_STATS
# builds (bound off / on), then whole-table times of the shipped library against
# build_ab/base (SPE_SETTLE=0), alternating.
#   bash tools/build_variant.sh base -DSPE_SETTLE=0
#   bash tools/build_variant.sh stats0 -DSPE_SETTLE=0 -DSPE_RELAX_STATS=1
#   bash tools/build_variant.sh stats1 -DSPE_SETTLE=1 -DSPE_RELAX_STATS=1
set -e
O=gpurun_out/settle_ab; mkdir -p $O
for V in stats0 stats1; do
  SPE_LIB=build_ab/$V/libspe.so timeout -k 10 200 python -u tools/exp_c3_stats.py > $O/$V.log 2>&1 || { tail -20 $O/$V.log; exit 1; }
  echo "stats $V: $(grep -c spe-relax-stats $O/$V.log) round lines"
done
run() {  # name, env...
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c3 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "frac", l["roofline"]["frac"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  run base SPE_LIB=build_ab/base/libspe.so
  run settle SPE_NOTHING=1
done
