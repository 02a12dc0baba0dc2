# Shared anchor trees on C4: rows-kernel variants (build_ab/) and the rows /
# relaxation overlap off, alternating, two passes.
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
  run cache X=1
  run nocache SPE_LIB=build_ab/nocache/libspe.so
  run cache_noovl SPE_NO_OVERLAP=1
  run nocache_noovl SPE_NO_OVERLAP=1 SPE_LIB=build_ab/nocache/libspe.so
done
