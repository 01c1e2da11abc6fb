# C4 N=1 with three engines taking the windows in turn (memory check first)
set -e
TAG=${1:-r04_d3}
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python bench.py --pipeline 3 --steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
echo done
