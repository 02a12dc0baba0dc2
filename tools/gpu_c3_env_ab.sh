# C3 A/B over environment settings of the Python mirror (SPE_INFL / SPE_OCC / ...)
set -e
O=gpurun_out/c3_env_ab; mkdir -p $O
run() {
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c3 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  run base SPE_NOTHING=1
  run i4o8 SPE_INFL=4 SPE_OCC=8
  run i6o6 SPE_INFL=6 SPE_OCC=6
done
