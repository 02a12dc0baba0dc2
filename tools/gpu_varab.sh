# same-box A/B of variant libraries ($VARIANTS, dirs with libspe.so) on C3 / C4, alternating
set -e
O=gpurun_out/${TAG:-varab}; mkdir -p $O
for r in 1 2; do
  for V in ${VARIANTS}; do
    for C in ${CONFIGS:-c3 c4}; do
      LOG=$O/$(basename $V)_${C}_$r.log
      SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$(basename $V) $C run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'])"
    done
  done
done
