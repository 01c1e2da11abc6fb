set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04_g4_tests.log 2>&1 &&
bash tools/gpu/r04_sim.sh s3d2 8 "3" --pipeline 2 &&
bash tools/gpu/r04_sim.sh s3d3 8 "3" --pipeline 3 &&
bash tools/gpu/r04_sim.sh s3d4 8 "3" --pipeline 4 &&
bash tools/gpu/r04_sim.sh s3d2r0 8 "3" --pipeline 2 --reserved-cus 0
