# D=3 at N=1: staggered ingests vs not (A/B, short legs off)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-stag}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 300 python bench.py $A --no-stagger > gpurun_out/${T}_ns.json 2> gpurun_out/${T}_ns.log &&
timeout -k 10 300 python bench.py $A > gpurun_out/${T}_s.json 2> gpurun_out/${T}_s.log &&
timeout -k 10 300 python bench.py $A --no-stagger > gpurun_out/${T}_ns2.json 2> gpurun_out/${T}_ns2.log
echo done
