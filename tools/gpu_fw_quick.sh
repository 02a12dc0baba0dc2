# FW engine parity + C2 FW bench line; then the N = 2 bench path rehearsed on one GPU (gloo, never for numbers)
set -e
O=gpurun_out/${TAG:-fwq}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fw_engine.py tests/test_gpu_fw.py tests/test_multi_device.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -60 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u bench.py --config c2fw > $O/bench_c2fw.log 2>&1 || { tail -20 $O/bench_c2fw.log; exit 1; }
tail -1 $O/bench_c2fw.log | cut -c1-900
SPE_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/rehearse_n2.log 2>&1 || { tail -30 $O/rehearse_n2.log; exit 1; }
grep '^{' $O/rehearse_n2.log | tail -1 | cut -c1-600
