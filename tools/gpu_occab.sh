# same-box: base vs variant at the compiler's occupancy vs SPE_OCC=$OCC (C3)
set -e
O=gpurun_out/${TAG:-occab}; mkdir -p $O
for r in 1 2; do
  for V in ${VARIANTS}; do
    for OC in 0 ${OCC:-5}; do
      LOG=$O/$(basename $V)_occ${OC}_$r.log
      SPE_OCC=$OC SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config ${CONF:-c3} --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$(basename $V) occ $OC run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'])"
    done
  done
done
