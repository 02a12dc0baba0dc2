# Shared anchor trees on C4: root capacity per batch (--groups = 64-lane blocks of
# roots; the one-GPU bench builds the whole table in one call), two passes.
set -e
O=gpurun_out/share_ab; mkdir -p $O
for rep in 1 2; do
  for G in ${GROUPS_LIST:-40 80 160 400}; do
    timeout -k 10 300 python -u bench.py --config c4 --groups $G --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_g${G}_$rep.log 2>&1 || { tail -20 $O/b_g${G}_$rep.log; exit 1; }
    python - $O/b_g${G}_$rep.log "c4 groups=$G rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r=l["roofline"]
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "frac", r["frac"], "lanes", r.get("relaxed_lanes_per_step"), "rounds", l["relax_rounds_per_step"], "kernel_ms", l["kernel_ms"], "launches", l["kernel_launches"]["init"])
PY
  done
done
