# FW engine parity (incl. multi-device and source trees) + the C2 FW bench line
set -e
O=gpurun_out/${TAG:-fwt}; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fw_engine.py tests/test_multi_device.py tests/test_gpu_source_tree.py -x -q --timeout 300 --timeout-method thread > $O/p.log 2>&1 || { tail -40 $O/p.log; exit 1; }
tail -1 $O/p.log
timeout -k 10 300 python -u bench.py --config c2fw --steps 2 > $O/b.log 2>&1 || { tail -20 $O/b.log; exit 1; }
grep '^{' $O/b.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['full_table_time_s'], d['closure_triple_s'], d['fw_kernels_ms_in_table_build'])"
