# derived-rows parity tests, the C3 default bench line, then the full-size C3 derived-rows parity test
set -e
O=gpurun_out/${TAG:-c3}
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
timeout -k 10 400 python -u bench.py --config c3 --steps ${STEPS:-3} --warmup 1 --no-side --cpu-seconds 2 --cpu-sources 0 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
if [ -n "$PARITY" ]; then
  timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_configs.py -k "c3_derived" -v -s --timeout 500 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
  grep -E "derived rows|passed|failed" $O/parity.log | tail -3
fi
