# Same-box A/B of env settings on one config: ENVS="A=1+B=2 C=3 ..." ("-" = no extra env), alternating twice
set -e
O=gpurun_out/${TAG:-envab}; mkdir -p $O
for r in 1 2; do
  for X in ${ENVS}; do
    EX=""; [ "$X" != "-" ] && EX=$(echo "$X" | tr '+' ' ')
    LOG=$O/$(echo "$X" | tr '+=' '__')_$r.log
    env $EX timeout -k 10 300 python -u bench.py --config ${CONFIG:-c3} --no-cpu-baseline --steps ${STEPS:-2} > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
    python -c "import json;d=json.loads(open('$LOG').read().strip().splitlines()[-1]);print('$X run $r', d['value'], d['ms_per_step'])"
  done
done
