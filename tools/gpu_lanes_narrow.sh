# C3 / C4 at lane widths 16 / 32 / 64 / 128 (same box)
set -e
O=gpurun_out/${TAG:-lanesn}; mkdir -p $O
for r in 1 2; do
  for W in ${WIDTHS:-16 32 64 128}; do
    for C in ${CONFIGS:-c3 c4}; do
      LOG=$O/L${W}_${C}_$r.log
      SPE_LANES=$W timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('L$W $C run $r', d['value'], d['full_table_time_s'], d['kernel_ms']['relax'], d['config'].get('groups_per_launch'))"
    done
  done
done
