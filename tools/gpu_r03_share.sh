# Round 3: shared anchor trees -- their parity file, the exact-mode pendant / parity
# files, the C4 bench both ways (default vs SPE_EXACT_SOURCES=1), the full-size C4 check.
set -e
O=gpurun_out/r03_share; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_shared_trees.py > $O/pytest_share.log 2>&1 || { tail -60 $O/pytest_share.log; exit 1; }
tail -1 $O/pytest_share.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_pendants.py tests/test_gpu_source_tree.py tests/test_gpu_contraction.py > $O/pytest_exact.log 2>&1 || { tail -40 $O/pytest_exact.log; exit 1; }
tail -1 $O/pytest_exact.log
for rep in 1 2; do
  for V in 0 1; do
    SPE_EXACT_SOURCES=$V timeout -k 10 300 python -u bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_c4_ex${V}_$rep.log 2>&1 || { tail -20 $O/b_c4_ex${V}_$rep.log; exit 1; }
    python - $O/b_c4_ex${V}_$rep.log "c4 exact_sources=$V rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r=l["roofline"]
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "avg_us", r["launch_avg_us"], "frac", r["frac"], "lanes", r.get("relaxed_lanes_per_step"), "rounds", l["relax_rounds_per_step"], "kernel_ms", l["kernel_ms"], "launches", l["kernel_launches"])
PY
  done
done
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o c4 -- python3 bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/prof_c4.log 2>&1 || { tail -20 $O/prof_c4.log; exit 1; }
find $O/prof_c4 -name "*kernel_stats.csv" | head -1 | xargs -I{} python -c "
import csv,sys
for r in list(csv.DictReader(open(sys.argv[1])))[:10]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])" {}
timeout -k 10 900 python -u -m pytest -x -q --timeout 800 --timeout-method thread tests/test_gpu_bench_configs.py -k c4 > $O/pytest_c4.log 2>&1 || { tail -30 $O/pytest_c4.log; exit 1; }
tail -1 $O/pytest_c4.log
