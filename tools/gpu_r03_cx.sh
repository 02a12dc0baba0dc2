# Round 3: degree-3 contraction -- its parity file, the whole parity suite at 128
# lanes, the full-size C3 / C4 configs, then a same-box A/B (SPE_NO_CONTRACT=1).
set -e
O=gpurun_out/r03_cx; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_contraction.py > $O/pytest_cx.log 2>&1 || { tail -40 $O/pytest_cx.log; exit 1; }
tail -1 $O/pytest_cx.log
SPE_LANES=128 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $O/pytest_parity128.log 2>&1 || { tail -30 $O/pytest_parity128.log; exit 1; }
tail -1 $O/pytest_parity128.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_gpu_bench_configs.py -k "c3 or c4" > $O/pytest_configs.log 2>&1 || { tail -30 $O/pytest_configs.log; exit 1; }
tail -1 $O/pytest_configs.log
for rep in 1 2; do
  for V in 0 1; do
    for C in c3 c4; do
      SPE_NO_CONTRACT=$V timeout -k 10 240 python -u bench.py --config $C --steps 2 --warmup 1 --no-cpu-baseline --no-side > $O/b_${C}_nc${V}_$rep.log 2>&1 || { tail -20 $O/b_${C}_nc${V}_$rep.log; exit 1; }
      python - $O/b_${C}_nc${V}_$rep.log "$C no_contract=$V rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
r=l["roofline"]
print(sys.argv[2], "table_s", l["full_table_time_s"], "src/s", l["value"], "avg_us", r["launch_avg_us"], "frac", r["frac"], "rounds", l["relax_rounds_per_step"], "kernel_ms", l["kernel_ms"])
PY
    done
  done
done
