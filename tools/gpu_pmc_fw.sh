# FETCH_SIZE / WRITE_SIZE passes (separate runs) of the FW engine's C2 bench -> profiles/r02_pmc_c2fw.json
set -e
O=gpurun_out/${TAG:-pmcfw}; mkdir -p $O
export TMPDIR=/tmp
A="--config c2fw --steps 1"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_c2fw -o run --output-format csv -- python bench.py $A > $O/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_c2fw -o run --output-format csv -- python bench.py $A > $O/pmc_write.log 2>&1
mkdir -p $O/pmc_c2fw && cp -r $O/pmc_fetch_c2fw $O/pmc_write_c2fw $O/pmc_c2fw/
python tools/pmc_to_json.py $O/pmc_c2fw profiles/r02_pmc_c2fw.json
