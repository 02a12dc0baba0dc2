# Round 6: the GPU suite on the shipped library (online margin proof + host single
# reads), then C3 / C4 whole tables against build_ab/base (SPE_MARGIN_ONLINE=0:
# k_share_check), alternating, and the drop-in lines.
#   bash tools/build_variant.sh base -DSPE_MARGIN_ONLINE=0
set -e
O=gpurun_out/r06_margin; mkdir -p $O
timeout -k 10 150 ./build_ab/probe_single_call > $O/probe.txt 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {  # name config env...
  N=$1; C=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-side > $O/b_${C}_${N}_$rep.log 2>&1 || { tail -20 $O/b_${C}_${N}_$rep.log; exit 1; }
  python - $O/b_${C}_${N}_$rep.log "$C $N rep=$rep" <<'PY'
import json,sys
l=json.loads([x for x in open(sys.argv[1]) if x.startswith("{")][-1])
print(sys.argv[2], "table_s", l["full_table_time_s"], "frac", l["roofline"]["frac"], "fallback", l["roofline"]["fallback_blocks_per_step"], "kernel_ms", {k: v for k, v in l["kernel_ms"].items() if v})
PY
}
for rep in 1 2; do
  run base c3 SPE_LIB=build_ab/base/libspe.so
  run online c3 SPE_NOTHING=1
done
run base c4 SPE_LIB=build_ab/base/libspe.so
run online c4 SPE_NOTHING=1
timeout -k 10 200 python -u bench.py --config c4shim --steps 2 --cpu-seconds 2 --queries 20000000 > $O/c4shim.out 2> $O/c4shim.err
timeout -k 10 200 python -u bench.py --config c3shim --steps 3 --cpu-seconds 2 --queries 20000000 > $O/c3shim.out 2> $O/c3shim.err
python - <<'PY'
import json
for c in ("c3shim", "c4shim"):
    l = json.loads(open(f"gpurun_out/r06_margin/{c}.out").read().strip().splitlines()[-1])
    print(c, "value", l["value"], "single", l["single_call_queries_per_s"], "startup", l["startup_s"])
PY
