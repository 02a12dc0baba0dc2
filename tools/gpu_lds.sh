# LDS engine check: full GPU parity suite (both engines), phase clocks, then C2 bench on each engine
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
SPE_LDS_DEBUG=1 timeout -k 10 300 python -u bench.py --config c2 --engine 2 --no-cpu-baseline --no-profile --steps 2 --warmup 0 > gpurun_out/c2_dbg.log 2>&1 || { tail -20 gpurun_out/c2_dbg.log; exit 1; }
grep spe-lds gpurun_out/c2_dbg.log | tail -1
for E in ${ENGINES:-2}; do
  timeout -k 10 300 python -u bench.py --config c2 --engine $E --no-cpu-baseline > gpurun_out/c2_e$E.log 2>&1 || { tail -20 gpurun_out/c2_e$E.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c2_e$E.log').read().strip().splitlines()[-1]);print('E=$E', d['value'], d['full_table_time_s'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['roofline']['frac'])"
done
