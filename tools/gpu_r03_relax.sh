# Round 3: parity of every relaxation shape, then a same-box A/B of the 128-lane
# relaxation kernels on C3 and C4 (whole tables, HIP-event launch times).
set -e
O=gpurun_out/r03_relax; mkdir -p $O
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "lane_group_widths or unbuilt or tie or directed" > $O/pytest_shapes.log 2>&1 || { tail -30 $O/pytest_shapes.log; exit 1; }
  tail -2 $O/pytest_shapes.log
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_multi_device.py > $O/pytest_multi.log 2>&1 || { tail -30 $O/pytest_multi.log; exit 1; }
  tail -2 $O/pytest_multi.log
fi
for rep in 1 2; do
IFS=';' read -ra VS <<< "${VARIANTS:-1,2,6;2,4,8;2,4,1;2,6,6;2,8,0}"
for V in "${VS[@]}"; do
  IFS=, read -r K1 K2 K3 <<< "$V"
  set -- $K1 $K2 $K3
  for C in c3 c4; do
    SPE_RELAX=$1 SPE_INFL=$2 SPE_OCC=$3 timeout -k 10 240 python -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_${C}_$1_$2_$3_$rep.log 2>&1 || { tail -20 $O/b_${C}_$1_$2_$3_$rep.log; exit 1; }
    python - $O/b_${C}_$1_$2_$3_$rep.log "$C relax=$1 rows=$2 occ=$3 rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r=l["roofline"]
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], r["kernel"], "avg_us", r["launch_avg_us"], "launches", r["launches"], "frac", r["frac"], "rounds", l["relax_rounds_per_step"])
PY
  done
done
done
