# parity suite, C5 lookups, C3 bench (no CPU leg)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -u bench.py --config c5 --steps 10 --warmup 2 > gpurun_out/c5.log 2>&1 || { tail -20 gpurun_out/c5.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c5.log').read().strip().splitlines()[-1]);print('C5', d['value']/1e9, 'Gq/s', d['roofline']['achieved'], d['ms_per_step'])"
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/c3.log 2>&1 || { tail -20 gpurun_out/c3.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/c3.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['full_table_time_s'], d['kernel_ms'])"
