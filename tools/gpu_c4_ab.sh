# C4 A/B over experimental libraries in build_ab/ (SPE_LIB), shipped library as "base"
set -e
O=gpurun_out/c4_ab; mkdir -p $O
run() {
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c4 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  run base SPE_NOTHING=1
  for V in $VARIANTS; do run $V SPE_LIB=build_ab/$V/libspe.so; done
done
