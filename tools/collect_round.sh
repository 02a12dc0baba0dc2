# copy the judged artefacts of a tools/gpu_profiles.sh run (+ gpu_tests.sh) into profiles/
set -e
R=${ROUND:-r04}
O=gpurun_out/$R
for C in c1 c2 c3 c4 c5 c5_on_c4 c2fw; do
  [ -f $O/bench_$C.log ] && tail -1 $O/bench_$C.log > profiles/${R}_bench_$C.json
  if [ -d $O/kt_$C ]; then
    f=$(find $O/kt_$C -name '*kernel_stats.csv' | head -1)
    if [ -n "$f" ]; then cp "$f" profiles/${R}_rocprof_kernel_stats_$C.csv; fi
  fi
  [ -d $O/pmc_$C ] && python tools/pmc_to_json.py $O/pmc_$C profiles/${R}_pmc_$C.json > /dev/null
done
ls profiles | grep "^$R"
