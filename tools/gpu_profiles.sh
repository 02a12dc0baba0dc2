# Round profiles: per config, separate FETCH_SIZE / WRITE_SIZE PMC passes
# (MI355X_MICROARCH.md HBM section) -> profiles/${R}_pmc_<config>.json on the box,
# then rocprofv3 kernel-trace stats of the same command, then the bench line itself
# (which reads the PMC summary back as roofline.traffic).
# Configs: c3 c2 c4 c5 (on the C3 table) c5_on_c4 (on the C4 table) c1 c2fw c3_exact c4_exact.
set -e
R=${ROUND:-r06}
O=gpurun_out/$R
mkdir -p $O
export TMPDIR=/tmp
args() {
  case $1 in
    c5) echo "--config c5 --steps 4 --warmup 1 --no-cpu-baseline" ;;
    c5_on_c4) echo "--config c5 --c5-table c4 --steps 4 --warmup 1 --no-cpu-baseline" ;;
    c2fw) echo "--config c2fw --steps 1" ;;
    c1) echo "--config c1 --steps 20 --warmup 2 --no-cpu-baseline --no-side" ;;
    c3_exact) echo "--config c3 --exact --no-compare --steps 2 --warmup 1 --no-cpu-baseline --no-side" ;;
    c4_exact) echo "--config c4 --exact --no-compare --steps 2 --warmup 1 --no-cpu-baseline --no-side" ;;
    *) echo "--config $1 --steps 2 --warmup 1 --no-cpu-baseline --no-side" ;;
  esac
}
for C in ${CONFIGS:-c3 c4 c1 c5_on_c4 c2 c5 c2fw}; do
  A=$(args $C)
  if [ -z "$NO_PMC" ]; then
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$C -o run --output-format csv -- python bench.py $A > $O/pmc_fetch_$C.log 2>&1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$C -o run --output-format csv -- python bench.py $A > $O/pmc_write_$C.log 2>&1
    mkdir -p $O/pmc_$C && cp -r $O/pmc_fetch_$C $O/pmc_write_$C $O/pmc_$C/
    python tools/pmc_to_json.py $O/pmc_$C profiles/${R}_pmc_$C.json $O/pmc_fetch_$C.log > /dev/null
    cp profiles/${R}_pmc_$C.json $O/   # only gpurun_out/ comes back from the box
  fi
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_$C -o run --output-format csv -- python bench.py $A > $O/kt_$C.log 2>&1
  timeout -k 10 300 python -u bench.py $A > $O/bench_$C.log 2>&1
  echo "profiled $C: $(tail -1 $O/bench_$C.log | cut -c1-160)"
done
