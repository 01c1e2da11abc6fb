# PMC passes (FETCH_SIZE, WRITE_SIZE: separate runs) of a short C4 bench, C5 leg off, for the
# replay's HBM traffic; the bench line of the same command gives the algorithmic bytes
set -e
TAG=${1:-r04_pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
A="--steps 1 --warmup 0 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --parity-keys 64"
timeout -k 10 300 python bench.py $A > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_fetch -o run -- python bench.py $A > gpurun_out/${TAG}_fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_write -o run -- python bench.py $A > gpurun_out/${TAG}_write.log 2>&1
echo done
