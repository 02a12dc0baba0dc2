# L2 engine: parity on every GPU test (engine l2 only), then C3 / C2 bench lines on it
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -k "l2" -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_l2.log 2>&1 || { tail -40 gpurun_out/pytest_l2.log; exit 1; }
tail -1 gpurun_out/pytest_l2.log
for C in ${CONFIGS:-c3 c2}; do
  timeout -k 10 200 python -u bench.py --config $C --engine 3 --steps ${STEPS:-4} --warmup 1 --no-cpu-baseline > gpurun_out/l2_$C.log 2>&1 || { tail -20 gpurun_out/l2_$C.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/l2_$C.log').read().strip().splitlines()[-1]);print('$C', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['roofline']['frac'])"
done
