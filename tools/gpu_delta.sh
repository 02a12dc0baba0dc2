# Delta-stepping schedule: parity tests, then the C3 (and C4) whole table at several Delta values
# beside the default Gauss-Seidel schedule (same box, alternating)
set -e
O=gpurun_out/${TAG:-delta}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_delta.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for D in 0 10 40 0 150 600; do
  if [ $D = 0 ]; then unset SPE_DELTA; else export SPE_DELTA=$D; fi
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-side > $O/c3_d$D.log 2>&1 || { tail -20 $O/c3_d$D.log; exit 1; }
  python -c "import json,sys; d=json.loads([l for l in open('$O/c3_d$D.log') if l.startswith('{')][-1]); print('C3 delta=$D', d['value'], d['full_table_time_s'], d['relax_rounds_per_step'], d['roofline']['launch_avg_us'], d['kernel_ms'])"
done
unset SPE_DELTA
