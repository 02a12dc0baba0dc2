# same-box A/B of the FW engine on C2 (variant dirs with libspe.so; in-tree FW parity first)
set -e
O=gpurun_out/${TAG:-fwab}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_fw_engine.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for V in ${VARIANTS:-build_A build_B}; do
    LOG=$O/${V}_$r.log
    SPE_LIB=$PWD/$V/libspe.so timeout -k 10 300 python -u bench.py --config c2fw --steps 2 > $LOG 2>&1 || { tail -5 $LOG; exit 1; }
    python -c "import json;d=json.loads([l for l in open('$LOG') if l.startswith('{')][-1]);print('$V run $r', d['full_table_time_s'], d['closure_triple_s'], d['closure_distance_only_s'])"
  done
done
