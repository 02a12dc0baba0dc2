# parity tests, then k_relax at the compiler's occupancy and forced variants (SPE_OCC)
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for O in ${OCCS:-0 7}; do
  SPE_OCC=$O timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline > gpurun_out/occ_$O.log 2>&1 || { tail gpurun_out/occ_$O.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/occ_$O.log').read().strip().splitlines()[-1]);print('OCC=$O', d['value'], d['kernel_ms'], d['relax_rounds_per_step'], d['roofline']['launch_avg_us'])"
  SPE_OCC=$O timeout -k 10 200 python -u bench.py --config c4 --full-table > gpurun_out/occ_c4_$O.log 2>&1 || { tail gpurun_out/occ_c4_$O.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/occ_c4_$O.log').read().strip().splitlines()[-1]);print('OCC=$O C4 full', d['value'], d['roofline']['frac'])"
done
