# four engines in turn on the hottest-key rank of N = 2, 4 and on other ranks of N = 8 (simulated per rank)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-ds}
bash tools/gpu/r04_sim.sh ${T}_p4 2 "1 0" --pipeline 4 &&
bash tools/gpu/r04_sim.sh ${T}_p4 4 "3 0" --pipeline 4 &&
bash tools/gpu/r04_sim.sh ${T}_p4 8 "0 5" --pipeline 4
echo "rc=$?"
