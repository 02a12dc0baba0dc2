# Parity tests at each lane-group width, then a C3 bench sweep over widths.
set -e
mkdir -p gpurun_out
for L in ${LS:-16 32 64}; do
  SPE_LANES=$L timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_L$L.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_L$L.log; exit 1; }
  echo "L=$L $(tail -1 gpurun_out/pytest_gpu_L$L.log)"
done
for L in ${LS:-16 32 64}; do
  for G in ${GS:-16}; do
    SPE_LANES=$L timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --groups $G --no-cpu-baseline > gpurun_out/lanes_L${L}_G$G.log 2>&1
    python -c "import json;d=json.loads(open('gpurun_out/lanes_L${L}_G$G.log').read().strip().splitlines()[-1]);print('L=$L G=$G', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
  done
done
