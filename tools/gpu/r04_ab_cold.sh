# A/B: the exact mode's one-wave replays on the normal-priority replay stream (VN_COLD_ST3) vs the main stream
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-cold}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for i in 1 2; do
  VN_COLD_ST3=1 timeout -k 10 300 python bench.py $A > gpurun_out/${T}_on$i.json 2> gpurun_out/${T}_on$i.log || exit 1
  timeout -k 10 300 python bench.py $A > gpurun_out/${T}_off$i.json 2> gpurun_out/${T}_off$i.log || exit 1
done
echo "rc=0"
