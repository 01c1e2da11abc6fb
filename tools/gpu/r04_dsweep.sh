# engines in turn (D) at N=1 and on the hottest-key rank of N = 2, 4, 8 (simulated per rank)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-ds}
bash tools/gpu/r04_ab_d4.sh ${T} &&
for D in 2 3 4; do
  bash tools/gpu/r04_sim.sh ${T}_p$D 8 "3" --pipeline $D || exit 1
done &&
for D in 2 3; do
  bash tools/gpu/r04_sim.sh ${T}_p$D 2 "1" --pipeline $D && bash tools/gpu/r04_sim.sh ${T}_p$D 4 "3" --pipeline $D || exit 1
done
echo "rc=$?"
