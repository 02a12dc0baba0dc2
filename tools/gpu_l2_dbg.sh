# L2 engine per-phase clocks (SPE_LDS_DEBUG) over configs and workgroup counts
set -e
mkdir -p gpurun_out
for C in ${CONFIGS:-c3 c2}; do
  for GR in ${GRIDS:-256}; do
    SPE_L2_GRID=$GR SPE_LDS_DEBUG=1 timeout -k 10 200 python -u bench.py --config $C --engine 3 --no-cpu-baseline --no-profile --steps 1 --warmup 0 > gpurun_out/l2dbg_$C.log 2>&1 || { tail -20 gpurun_out/l2dbg_$C.log; exit 1; }
    echo "$C grid=$GR $(grep spe-l2 gpurun_out/l2dbg_$C.log | tail -1)"
    SPE_L2_GRID=$GR timeout -k 10 200 python -u bench.py --config $C --engine 3 --no-cpu-baseline --steps 2 --warmup 1 > gpurun_out/l2b_$C.log 2>&1 || { tail -20 gpurun_out/l2b_$C.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/l2b_$C.log').read().strip().splitlines()[-1]);print('  $C grid=$GR', d['value'], 'sources/s', d['roofline']['launch_avg_us'])"
  done
done
