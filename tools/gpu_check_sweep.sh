# Parity tests + groups-per-launch sweep on C3 (cache-residency experiment).
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for G in ${GS:-1 2 4 16}; do
  timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --groups $G --no-cpu-baseline > gpurun_out/sweep_g$G.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/sweep_g$G.log').read().strip().splitlines()[-1]);print('G=$G', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
