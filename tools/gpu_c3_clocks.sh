# C3 box modes vs the clocks the GPU runs at DURING the tables (rocm-smi sampled
# every ~0.5 s in the background): six processes, eight timed tables each.
set -e
O=gpurun_out/${TAG:-c3clk}; mkdir -p $O
for r in 1 2 3 4 5 6; do
  ( for i in $(seq 60); do rocm-smi --showclocks 2>/dev/null | grep -E "fclk|mclk|sclk|socclk" | tr '\n' ' '; echo; sleep 0.5; done ) > $O/clk$r.txt &
  P=$!
  timeout -k 10 300 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline --no-side --no-profile > $O/run$r.log 2>&1 || { kill $P; tail -20 $O/run$r.log; exit 1; }
  kill $P 2>/dev/null || true
  wait $P 2>/dev/null || true
  python - $O/run$r.log $O/clk$r.txt $r <<'PY'
import json,sys,re,collections
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
c=collections.Counter()
for line in open(sys.argv[2]):
    for k,v in re.findall(r"(\w+) clock level: \d+: \((\d+)Mhz\)", line): c[(k,v)]+=1
print("run", sys.argv[3], "step_s", min(l["rank0_step_s"]), max(l["rank0_step_s"]), dict(c))
PY
done
