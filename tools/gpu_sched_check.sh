# bench at N = 1 and the N = 2 path rehearsed on one GPU (gloo; never for numbers)
set -e
O=gpurun_out/${TAG:-sched}; mkdir -p $O
timeout -k 10 300 python -u bench.py --steps 1 --no-cpu-baseline --no-side > $O/n1.log 2>&1 || { tail -20 $O/n1.log; exit 1; }
tail -1 $O/n1.log | cut -c1-300
SPE_BENCH_REHEARSE_ONE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 1 --warmup 1 --no-cpu-baseline > $O/n2.log 2>&1 || { tail -30 $O/n2.log; exit 1; }
grep '^{' $O/n2.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['chunk_schedule'], d['gather_bytes_per_gpu_per_step'], d['value'])"
