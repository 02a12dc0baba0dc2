# Round 6: k_rows_lm XCD mapping A/B on C3 (shipped: XCD = eighth of the source blocks;
# build_ab/base: eighth of the target tiles), alternating, then a PMC pass of each.
set -e
O=gpurun_out/r06_rows; mkdir -p $O
export TMPDIR=/tmp
run() {  # name env...
  N=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline --no-side > $O/b_${N}_$rep.log 2>&1 || { tail -20 $O/b_${N}_$rep.log; exit 1; }
  python - $O/b_${N}_$rep.log "c3 $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2 3; do
  run base SPE_LIB=build_ab/base/libspe.so
  run xcdblk SPE_NOTHING=1
done
for N in base xcdblk; do
  L=""; [ $N = base ] && L=build_ab/base/libspe.so
  SPE_LIB=$L timeout -s KILL 200 rocprofv3 --kernel-trace --stats -d $O/kt_$N -o run --output-format csv -- python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/kt_$N.log 2>&1
  SPE_LIB=$L timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $O/pf_$N -o run --output-format csv -- python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/pf_$N.log 2>&1
  python - $O/pf_$N $N <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(float); nd = collections.defaultdict(set)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0].replace("void ", "")
        acc[k] += float(r["Counter_Value"]); nd[k].add(r["Dispatch_Id"])
for k in ("k_rows_lm", "k_stage_lanes", "k_relax_s"):
    print(sys.argv[2], k, "fetch GB per dispatch (x2 gfx950):", round(2 * acc[k] * 1024 / max(1, len(nd[k])) / 1e9, 2))
PY
  f=$(find $O/kt_$N -name '*kernel_stats.csv' | head -1); grep -E "k_rows_lm|k_stage_lanes" "$f" | cut -d, -f1-4 | sed 's/(anonymous namespace):://g' | cut -c1-40,200-
done
