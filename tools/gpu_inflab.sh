# same-box: rows in flight (SPE_INFL) and forced occupancy (SPE_OCC) of k_relax_m at 128 lanes, C3 / C4
# LIST: infl_occ pairs (occ 0 = the compiler's choice)
set -e
O=gpurun_out/${TAG:-inflab}; mkdir -p $O
for r in ${RUNS:-1 2}; do
  for V in ${LIST:-4_0 3_0 2_0 2_6}; do
    I=${V%_*}; OC=${V#*_}
    for C in ${CONFIGS:-c3 c4}; do
      LOG=$O/i${I}_o${OC}_${C}_$r.log
      SPE_INFL=$I SPE_OCC=$OC timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('infl $I occ $OC $C run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'])"
    done
  done
done
