set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python3 -u bench.py --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 --text-lines 0"
timeout -s KILL 600 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r03_v3_pmc_fetch -o f --output-format csv -- $B > gpurun_out/r03_v3_pmc_fetch.json 2> gpurun_out/r03_v3_pmc_fetch.log &&
timeout -s KILL 600 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r03_v3_pmc_write -o w --output-format csv -- $B > gpurun_out/r03_v3_pmc_write.json 2> gpurun_out/r03_v3_pmc_write.log
echo "rc=$?"
