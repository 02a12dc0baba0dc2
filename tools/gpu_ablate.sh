set -e
mkdir -p gpurun_out
for A in 0 1; do
  SPE_ABLATE=$A timeout -k 10 200 python -u bench.py --steps 8 --warmup 1 --groups 16 --no-cpu-baseline > gpurun_out/abl_$A.log 2>&1 || { tail gpurun_out/abl_$A.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/abl_$A.log').read().strip().splitlines()[-1]);print('ABLATE=$A', d['value'], d['kernel_ms'], d['relax_rounds_per_step'])"
done
export TMPDIR=/tmp
B="python bench.py --steps 2 --warmup 0 --groups 16 --no-cpu-baseline --no-profile"
i=0
for set in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set -d gpurun_out/pmc2/p$i -o run --output-format csv -- $B > gpurun_out/pmc2_p$i.log 2>&1 || echo "pass $i failed"
done
python tools/pmc_summary.py gpurun_out/pmc2
