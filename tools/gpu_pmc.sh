# PMC passes over a short C3 bench (each pass its own rocprofv3 run, <= 8 SQ / 4 TCC counters)
set -e
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
B="python bench.py --steps 2 --warmup 0 --groups ${G:-16} --no-cpu-baseline --no-profile"
i=0
for set in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" \
           "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SMEM SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR" \
           "TA_BUSY_avr TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc/p$i -o run --output-format csv -- $B > gpurun_out/pmc/p$i.log 2>&1 || echo "pass $i failed: $set"
done
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt || true
cat gpurun_out/pmc/summary.txt
