# parity suite, then the C3 (batch engine) and C2 (LDS engine) bench lines
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for C in c3 c2; do
  timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline > gpurun_out/chk_$C.log 2>&1 || { tail -20 gpurun_out/chk_$C.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/chk_$C.log').read().strip().splitlines()[-1]);print('$C', d['value'], d['full_table_time_s'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['roofline']['frac'], d.get('relax_rounds_per_step'))"
done
