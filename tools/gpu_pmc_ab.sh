# PMC A/B of relaxation variants on one config: HBM bytes (FETCH_SIZE / WRITE_SIZE,
# separate passes), memory-side requests and wave wait share, per variant (SPE_RELAX
# values in $VARIANTS).  Summaries in gpurun_out/$TAG/<variant>/summary.txt.
set -e
O=gpurun_out/${TAG:-pmcab}; mkdir -p $O
export TMPDIR=/tmp
C=${CONFIG:-c3}
A="--config $C --steps 1 --warmup 0 --no-cpu-baseline --no-side --no-profile"
for V in ${VARIANTS:-2 3}; do
  D=$O/v$V; mkdir -p $D
  export SPE_RELAX=$V
  timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $D/p1 -o run --output-format csv -- python bench.py $A > $D/p1.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $D/p2 -o run --output-format csv -- python bench.py $A > $D/p2.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum -d $D/p3 -o run --output-format csv -- python bench.py $A > $D/p3.log 2>&1
  timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $D/p4 -o run --output-format csv -- python bench.py $A > $D/p4.log 2>&1
  python tools/pmc_summary.py $D > $D/summary.txt
  echo "== variant $V"; grep -A12 "k_relax_s" $D/summary.txt | head -14
done
