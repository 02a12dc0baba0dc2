# A/B of experimental libraries (build_ab/<name>/libspe.so via SPE_LIB; "base" =
# the shipped library) on one config: per variant the bench line (table time)
# and a rocprofv3 kernel-trace summary (per-kernel ms per table), REPS passes
# alternating the variants.  CONFIG (default c3), VARIANTS, REPS (default 2).
set -e
export TMPDIR=/tmp
C=${CONFIG:-c3}
O=gpurun_out/ab_$C; mkdir -p $O
STEPS=${STEPS:-3}
for rep in $(seq 1 ${REPS:-2}); do
  for V in base $VARIANTS; do
    if [ $V = base ]; then unset SPE_LIB; else export SPE_LIB=build_ab/$V/libspe.so; fi
    timeout -k 10 300 python -u bench.py --config $C --steps $STEPS --warmup 1 --no-cpu-baseline --no-side > $O/b_${V}_$rep.log 2>&1 || { tail -20 $O/b_${V}_$rep.log; exit 1; }
    if [ $rep = 1 ]; then
      timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_$V -o run --output-format csv -- python -u bench.py --config $C --steps $STEPS --warmup 1 --no-cpu-baseline --no-side > $O/kt_$V.log 2>&1 || { tail -20 $O/kt_$V.log; exit 1; }
    fi
    python tools/ab_summary.py $O $V $rep $((STEPS + 1))
  done
done
