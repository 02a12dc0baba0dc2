# PMC characterisation of the C3 relaxation kernel the bench ships (separate
# rocprofv3 --pmc passes within the per-block limits)
set -e
O=gpurun_out/${TAG:-pmcc}; mkdir -p $O
export TMPDIR=/tmp
A="--steps 1 --warmup 0 --no-cpu-baseline --no-side --no-profile"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES -d $O/p1 -o run --output-format csv -- python bench.py $A > $O/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TA_BUSY_avr TA_TA_BUSY_sum -d $O/p2 -o run --output-format csv -- python bench.py $A > $O/p2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $O/p3 -o run --output-format csv -- python bench.py $A > $O/p3.log 2>&1
python tools/pmc_summary.py $O > $O/summary.txt
cat $O/summary.txt
