# same-box: Voronoi cell size of spe_order_sources (SPE_ORDER_CELL) at the default lane width, C3 / C4
set -e
O=gpurun_out/${TAG:-cellab}; mkdir -p $O
for r in ${RUNS:-1 2}; do
  for CS in ${CELLS:-64 128 256}; do
    for C in ${CONFIGS:-c3 c4}; do
      LOG=$O/cell${CS}_${C}_$r.log
      SPE_ORDER_CELL=$CS timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('cell $CS $C run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'])"
    done
  done
done
