# parity tests, then C4 (step bench: rows kernel time) and the C4 full table, C3
set -e
mkdir -p gpurun_out/rows
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/rows/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/rows/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/rows/pytest_gpu.log
timeout -k 10 200 python -u bench.py --config c4 --steps 20 --warmup 2 --no-cpu-baseline > gpurun_out/rows/c4_steps.log 2>&1 || { tail gpurun_out/rows/c4_steps.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/rows/c4_steps.log').read().strip().splitlines()[-1]);print('C4 steps', d['value'], d['kernel_ms'], d['roofline_rows'])"
timeout -k 10 200 python -u bench.py --config c4 --full-table > gpurun_out/rows/c4_full.log 2>&1 || { tail gpurun_out/rows/c4_full.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/rows/c4_full.log').read().strip().splitlines()[-1]);print('C4 full', d['value'], d['roofline']['frac'])"
timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/rows/c3.log 2>&1 || { tail gpurun_out/rows/c3.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/rows/c3.log').read().strip().splitlines()[-1]);print('C3', d['value'], d['kernel_ms'])"
