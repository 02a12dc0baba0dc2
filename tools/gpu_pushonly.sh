# LDS-engine timing variants on C2 (dirs under build_ab/ with a libspe.so, e.g. built
# with -DSPE_LDS_PUSH_ONLY by tools/build_flags_variant.sh): one bench line each
O=gpurun_out/${TAG:-pushonly}; mkdir -p $O
for V in ${VARIANTS}; do
  SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config ${CONFIG:-c2} --no-cpu-baseline --steps 5 > $O/$(basename $V).log 2>&1 || { tail -5 $O/$(basename $V).log; exit 1; }
  python -c "import json;d=json.loads(open('$O/$(basename $V).log').read().strip().splitlines()[-1]);print('$V', d['value'], d['ms_per_step'])"
done
