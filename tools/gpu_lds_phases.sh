# LDS engine phase clocks (SPE_LDS_DEBUG) for the in-tree build and $VARIANTS (dirs with libspe.so)
set -e
O=gpurun_out/${TAG:-ldsph}
mkdir -p $O
for V in tree ${VARIANTS}; do
  if [ $V = tree ]; then unset SPE_LIB; else export SPE_LIB=$PWD/$V/libspe.so; fi
  SPE_LDS_DEBUG=1 timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline --steps 1 --warmup 0 > $O/ph_$(basename $V).log 2>&1 || { tail -20 $O/ph_$(basename $V).log; exit 1; }
  echo $V; grep spe-lds $O/ph_$(basename $V).log | tail -1
done
# lane-group width on C3 (SPE_LANES: 32 vs 64 sources per relaxation row)
for L in ${LANES}; do
  SPE_LANES=$L timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 2 > $O/c3_L$L.log 2>&1 || { tail -20 $O/c3_L$L.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/c3_L$L.log').read().strip().splitlines()[-1]);print('L=$L', d['value'], d['kernel_ms']['relax'], d['roofline']['launch_avg_us'], d['relax_rounds_per_step'])"
done
