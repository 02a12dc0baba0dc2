# Quick parity + C3 bench over relax variants given as "L:INFL:OCC" in VARS.
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
echo "parity: $(tail -1 gpurun_out/pytest_gpu.log)"
for V in ${VARS:-64:8:0}; do
  IFS=: read L I O <<< "$V"
  SPE_LANES=$L SPE_INFL=$I SPE_OCC=$O timeout -k 10 200 python -u bench.py --steps 6 --warmup 1 --groups ${G:-16} --config ${CFG:-c3} --no-cpu-baseline > gpurun_out/var_${L}_${I}_${O}.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/var_${L}_${I}_${O}.log').read().strip().splitlines()[-1]);print('$V', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
