# Lane-group width L (sources per relaxation row): parity at $PLANES, then bench $CONFIGS at $LANES.
# A LANES entry may carry extra env settings: "128+SPE_INFL=8+SPE_OCC=6".
set -e
O=gpurun_out/${TAG:-lanes}
mkdir -p $O
for L in ${PLANES}; do
  SPE_LANES=$L timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_gpu_parity.py ${PTESTS} > $O/parity_L$L.log 2>&1 || { tail -30 $O/parity_L$L.log; exit 1; }
  echo "parity L=$L: $(tail -1 $O/parity_L$L.log)"
done
for C in ${CONFIGS:-c3}; do
  for X in ${LANES}; do
    L=${X%%+*}
    EX=""
    case $X in *+*) EX=$(echo "${X#*+}" | tr '+' ' ');; esac
    LOG=$O/${C}_$(echo $X | tr '+=' '__').log
    env SPE_LANES=$L $EX timeout -k 10 300 python -u bench.py --config $C --no-cpu-baseline --steps ${STEPS:-2} > $LOG 2>&1 || { tail -20 $LOG; exit 1; }
    python -c "import json;d=json.loads(open('$LOG').read().strip().splitlines()[-1]);print('$C $X', d['value'], d['ms_per_step'], d['kernel_ms'].get('relax'), d['roofline']['launch_avg_us'], d.get('relax_rounds_per_step'))"
  done
done
