# Round 6: GPU suite, then the drop-in lines (c3shim / c4shim) on the shipped library.
set -e
O=gpurun_out/r06_shim; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for c in c4shim c3shim; do
  timeout -k 10 200 python -u bench.py --config $c --steps 2 --cpu-seconds 2 --queries 20000000 > $O/$c.out 2> $O/$c.err
done
python - <<'PY'
import json
for c in ("c3shim", "c4shim"):
    l = json.loads(open(f"gpurun_out/r06_shim/{c}.out").read().strip().splitlines()[-1])
    print(c, "value", l["value"], "single", l["single_call_queries_per_s"], "startup", l["startup_s"])
PY
