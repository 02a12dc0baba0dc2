# C3 whole-table time vs 64-source groups per launch (state working set vs MALL)
set -e
O=gpurun_out/${TAG:-gsweep}
mkdir -p $O
for G in ${GROUPS_LIST:-2 4 8 16 48}; do
  timeout -k 10 300 python -u bench.py --groups $G --steps 2 --warmup 1 --no-cpu-baseline > $O/c3_g$G.log 2>&1 || { tail -20 $O/c3_g$G.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/c3_g$G.log').read().strip().splitlines()[-1]);print('G=$G', d['value'], d['kernel_ms']['relax'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
