# same-box A/B: the in-tree libspe.so against $BASE/libspe.so (tools/build_variant.sh),
# alternating, C3 whole tables (+ C4 if CONFIGS says so)
set -e
O=gpurun_out/${TAG:-ab2}
mkdir -p $O
BASE=${BASE:-build_ab/base}
for C in ${CONFIGS:-c3}; do
  for i in 1 2; do
    for V in base new; do
      if [ $V = base ]; then export SPE_LIB=$PWD/$BASE/libspe.so; else unset SPE_LIB; fi
      timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps ${STEPS:-3} > $O/${C}_${V}_$i.log 2>&1 || { tail -20 $O/${C}_${V}_$i.log; exit 1; }
      python -c "import json;d=json.loads(open('$O/${C}_${V}_$i.log').read().strip().splitlines()[-1]);print('$C $V $i', d['value'], d['full_table_time_s'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
    done
  done
done
