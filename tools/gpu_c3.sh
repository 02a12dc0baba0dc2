# parity suite, then the C3 bench (full table, no CPU leg)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python -u bench.py --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/c3.log 2>&1 || { tail -20 gpurun_out/c3.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c3.log').read().strip().splitlines()[-1]);print(d['value'], d['full_table_time_s'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['roofline']['frac'], d['relax_rounds_per_step'])"
