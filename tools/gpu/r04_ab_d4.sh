# A/B: four engines in turn (per-class caps make them fit), HW queues 16 / 32, against three
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-d4}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 300 python bench.py $A --pipeline 4 > gpurun_out/${T}_d4.json 2> gpurun_out/${T}_d4.log &&
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py $A --pipeline 4 > gpurun_out/${T}_d4q32.json 2> gpurun_out/${T}_d4q32.log &&
timeout -k 10 300 python bench.py $A > gpurun_out/${T}_d3.json 2> gpurun_out/${T}_d3.log
echo "rc=$?"
