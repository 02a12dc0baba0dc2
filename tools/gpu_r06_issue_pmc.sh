# Round 6: is k_relax_s issue-bound?  Instruction counts and per-unit active cycles
# of the C3 relaxation (separate --pmc passes, 8 SQ counters at most each).
set -e
O=gpurun_out/r06_issue; mkdir -p $O
export TMPDIR=/tmp
A="--steps 1 --warmup 0 --no-cpu-baseline --no-side --no-profile --no-compare"
timeout -s KILL 60 rocprofv3 -L > $O/avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/avail.txt | sort -u > $O/sq_names.txt || true
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_BRANCH -d $O/p1 -o run --output-format csv -- python bench.py $A > $O/p1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/p2 -o run --output-format csv -- python bench.py $A > $O/p2.log 2>&1
python tools/pmc_summary.py $O > $O/summary.txt
grep -A20 "k_relax_s" $O/summary.txt | head -24
