# Shared anchor trees on C4: rows-kernel variants (build_ab/), overlap off, two passes.
set -e
O=gpurun_out/share_rows_ab; mkdir -p $O
run() {  # name, env...
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c4 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  for V in b16t4 b32t2 b16t8 b32t4 b16t2; do run $V SPE_LIB=build_ab/$V/libspe.so; done
done
