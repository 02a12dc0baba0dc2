# C3 whole-table time against the GPU's temperature / power / clocks, run after run
set -e
O=gpurun_out/${TAG:-c3therm}; mkdir -p $O
for r in 1 2 3 4 5 6 7 8; do
  rocm-smi --showtemp --showpower --showclocks > $O/smi_$r.txt 2>&1 || true
  timeout -k 10 300 python -u bench.py --steps 12 --warmup 1 --no-cpu-baseline --no-side --no-profile > $O/run$r.log 2>&1 || { tail -20 $O/run$r.log; exit 1; }
  python - $O/run$r.log $O/smi_$r.txt $r <<'PY'
import json,sys,re
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
smi=open(sys.argv[2]).read()
t=re.findall(r"Temperature \(Sensor (\w+)\) \(C\): ([\d.]+)", smi)
p=re.findall(r"Power \(W\): ([\d.]+)", smi)
print("run", sys.argv[3], "step_s min/max", min(l["rank0_step_s"]), max(l["rank0_step_s"]), "temps", t, "power", p)
PY
done
