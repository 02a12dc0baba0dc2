# LDS engine: parity tests, then the C2 bench line and the phase clocks
set -e
O=gpurun_out/${TAG:-lds}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "lds or c2 or parity or pendants or owner or complete" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $O/bench_c2.log 2>&1 || { tail -20 $O/bench_c2.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_c2.log').read().strip().splitlines()[-1]);print('C2', d['value'], d['full_table_time_s'], d['roofline']['frac'])"
SPE_LDS_DEBUG=1 timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 0 > $O/c2_phases.log 2>&1 || { tail -20 $O/c2_phases.log; exit 1; }
grep spe-lds $O/c2_phases.log | tail -2
