set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r04_sim.sh s2d1 8 "3" --pipeline 1 &&
bash tools/gpu/r04_sim.sh s2d2r0 8 "3" --pipeline 2 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s2d3 8 "3" --pipeline 3 &&
bash tools/gpu/r04_sim.sh s2d4 8 "3" --pipeline 4 &&
bash tools/gpu/r04_sim.sh s2d4r0 8 "3" --pipeline 4 --reserved-cus 0
