set -e
mkdir -p gpurun_out
run() { env "$@" timeout -k 10 120 python -u tools/exp_knobs.py 64 2>&1 | grep -v amdgpu.ids; }
run X=0
run SPE_INFL=12
run SPE_INFL=16
run SPE_OCC=7
run SPE_OCC=8
