# D=3 at N=1: CUs reserved for the longest replays (A/B, short legs off)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-res}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for r in 8 16 32; do
  timeout -k 10 300 python bench.py $A --reserved-cus $r > gpurun_out/${T}_r$r.json 2> gpurun_out/${T}_r$r.log || exit 1
done
echo done
