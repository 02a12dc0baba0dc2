# C3 run-to-run spread: several processes of 8 timed tables each, per-step times,
# with the GPU's clocks before and after (is the slow mode per process or per step?)
set -e
O=gpurun_out/${TAG:-c3modes}; mkdir -p $O
rocm-smi --showclocks > $O/clocks_before.txt 2>&1 || true
for r in 1 2 3 4; do
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-side > $O/run$r.log 2>&1 || { tail -20 $O/run$r.log; exit 1; }
  python - $O/run$r.log $r <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print("run", sys.argv[2], "steps", l["rank0_step_s"], "relax avg_us", l["roofline"]["launch_avg_us"], "rounds", l["relax_rounds_per_step"])
PY
done
rocm-smi --showclocks > $O/clocks_after.txt 2>&1 || true
cat $O/clocks_after.txt | grep -i "mclk\|sclk\|fclk" | head -8
