# same-box A/B of groups per build launch on C3 / C4 (alternating)
set -e
O=gpurun_out/${TAG:-grab}; mkdir -p $O
for r in 1 2; do
  for C in c3 c4; do
    for G in ${GROUPS_LIST:-0 262 392}; do
      LOG=$O/${C}_g${G}_$r.log
      timeout -k 10 300 python -u bench.py --config $C --groups $G --no-cpu-baseline --no-side --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
      python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$C groups=$G run $r', d['value'], d['full_table_time_s'], d['config']['chunk_blocks'], d['relax_rounds_per_step'])"
    done
  done
done
