# Round 6: the library's background pre-fault of the table's host mapping and the
# shim's reader-sharded state lock -- the drop-in tests, then the c4shim / c3shim lines.
# EXP=1 also runs the library-level diagnostic (tools/exp_host_reads_mt.py).
set -e
O=gpurun_out/r06_prefault; mkdir -p $O
if [ -n "$EXP" ]; then
  timeout -k 10 400 python -u tools/exp_host_reads_mt.py > $O/exp.log 2>&1 || { tail -20 $O/exp.log; exit 1; }
  cat $O/exp.log
fi
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_host_reads.py tests/test_topology_shim.py tests/test_topology_batch.py tests/test_topology_cache.py tests/test_gpu_complete.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for c in c4shim c3shim; do
  timeout -k 10 300 python -u bench.py --config $c --steps 2 --cpu-seconds 2 --queries 20000000 > $O/$c.out 2> $O/$c.err
done
python - <<'PY'
import json
for c in ("c3shim", "c4shim"):
    l = json.loads(open(f"gpurun_out/r06_prefault/{c}.out").read().strip().splitlines()[-1])
    print(c, "value", l["value"], "single", l["single_call_queries_per_s"], "startup", l["startup_s"])
    print("   C:", l["single_call_queries_per_s_c"])
PY
