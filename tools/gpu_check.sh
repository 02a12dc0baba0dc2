# parity suite (short form) then the C3 batch timing; stops at the first failure
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for K in X=0 ${KNOBS}; do env $K timeout -k 10 120 python -u tools/exp_knobs.py 64 2>&1 | grep -v amdgpu.ids; done
