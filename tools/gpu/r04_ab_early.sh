# A/B: top-first chunk sort with the top replays on their own stream vs the round-4 layout; HW queues
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-early}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
VN_NO_EARLY=1 timeout -k 10 300 python bench.py $A > gpurun_out/${T}_off.json 2> gpurun_out/${T}_off.log &&
timeout -k 10 300 python bench.py $A > gpurun_out/${T}_on.json 2> gpurun_out/${T}_on.log &&
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py $A > gpurun_out/${T}_on32.json 2> gpurun_out/${T}_on32.log &&
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python bench.py $A --pipeline 4 > gpurun_out/${T}_on32d4.json 2> gpurun_out/${T}_on32d4.log
echo "rc=$?"
