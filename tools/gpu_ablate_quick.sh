set -e
mkdir -p gpurun_out
for A in ${ABLATIONS:-0 1}; do
  SPE_ABLATE=$A timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --no-cpu-baseline > gpurun_out/abl_$A.log 2>&1 || { tail gpurun_out/abl_$A.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abl_$A.log').read().strip().splitlines()[-1]);print('ABLATE=$A', d['value'], d['kernel_ms'], d['relax_rounds_per_step'], d['roofline']['launch_avg_us'])"
done
