# C3 batch engine: sources per launch (groups of 64) sweep
set -e
mkdir -p gpurun_out
for G in ${GROUPS_LIST:-1 2 4 8 16}; do
  timeout -k 10 200 python -u bench.py --steps ${STEPS:-8} --warmup 1 --groups $G --blocks-per-step 16 --no-cpu-baseline > gpurun_out/grp_$G.log 2>&1 || { tail -20 gpurun_out/grp_$G.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/grp_$G.log').read().strip().splitlines()[-1]);print('G=$G', d['value'], d['kernel_ms'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
