# Round 6 close-out on one GPU: the full GPU suite, smoke, then the driver's default
# bench command (C3 + every side config) with the shim seals' phase timing on stderr.
set -e
O=gpurun_out/r06_final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
S=$(date +%s)
SHADOW_SPE_SEAL_TIMING=1 timeout -k 10 800 python -u bench.py > $O/bench.out 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s, line $(tail -1 $O/bench.out | wc -c) B"
cp gpurun_out/bench_full_n1.json $O/
