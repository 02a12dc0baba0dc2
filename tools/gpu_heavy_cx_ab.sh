# C3 (contracted): rows per round trip of the contracted heavy partial (build_ab/
# variants of SPE_HEAVY_CX_INFL), alternating, two passes.
set -e
O=gpurun_out/heavy_cx_ab; mkdir -p $O
run() {
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c3 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  run hx5 X=1
  for V in 2 3 4; do run hx$V SPE_LIB=build_ab/hx$V/libspe.so; done
done
