# LDS engine phase breakdown on C2 (diagnostic clocks, SPE_LDS_DEBUG)
set -e
mkdir -p gpurun_out
SPE_LDS_DEBUG=1 timeout -k 10 300 python -u bench.py --config c2 --engine 2 --no-cpu-baseline --no-profile --steps 2 --warmup 0 > gpurun_out/c2_dbg.log 2>&1 || { tail -20 gpurun_out/c2_dbg.log; exit 1; }
grep spe-lds gpurun_out/c2_dbg.log | tail -3
