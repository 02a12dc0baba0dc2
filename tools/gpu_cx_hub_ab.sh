# C3: degree-3 contraction keeping vertices next to hubs (build_ab/ variants), alternating, two passes.
set -e
O=gpurun_out/cx_hub_ab; mkdir -p $O
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
  run base X=1
  run hub40 SPE_LIB=build_ab/hub40/libspe.so
  run hub64 SPE_LIB=build_ab/hub64/libspe.so
  run hub200 SPE_LIB=build_ab/hub200/libspe.so
done
