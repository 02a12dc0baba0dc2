# quick A/B of the current build: batch-engine parity subset + C3 and C4 bench lines
set -e
O=gpurun_out/${TAG:-ab}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "parity or pendants or owner or bench_configs or complete" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for C in c3 c4; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps ${STEPS:-3} > $O/bench_$C.log 2>&1 || { tail -20 $O/bench_$C.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$C.log').read().strip().splitlines()[-1]);print('$C', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
