# PMC passes (one counter group each) of a short bench run, for the roofline kernel's HBM traffic
set -e
TAG=${1:-rXX}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${TAG}_pmcbench.json 2> gpurun_out/${TAG}_pmcbench.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- python bench.py --steps 1 --warmup 0 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${TAG}_pmc_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- python bench.py --steps 1 --warmup 0 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${TAG}_pmc_write.log 2>&1
