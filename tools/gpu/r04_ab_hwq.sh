# D=3 at N=1: hardware queues 16 vs 24 vs 32 (A/B, short legs off)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-hwq}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for q in 16 24 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py $A > gpurun_out/${T}_q$q.json 2> gpurun_out/${T}_q$q.log || exit 1
done
echo done
