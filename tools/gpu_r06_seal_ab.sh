# Round 6: c4shim seal time with and without the library's background pre-fault
# (SPE_HOST_PREFAULT=0 / default), twice each, alternating.
set -e
O=gpurun_out/r06_seal_ab; mkdir -p $O
for k in 1 2; do
  for pf in 0 1; do
    SPE_HOST_PREFAULT=$pf timeout -k 10 300 python -u bench.py --config c4shim --steps 2 --cpu-seconds 1 --queries 20000000 --no-cpu-baseline > $O/pf${pf}_$k.out 2> $O/pf${pf}_$k.err
    echo "pf=$pf run $k: $(grep -h 'seal\|single calls' $O/pf${pf}_$k.err | tr '\n' ' ' | cut -c1-600)"
  done
done
