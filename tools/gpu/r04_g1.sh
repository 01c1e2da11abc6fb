set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04_g1_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/r04_g1_hot.log 2>&1 &&
timeout -k 10 300 python -u tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/r04_g1_c5.log 2>&1 &&
bash tools/gpu/r04_e5.sh
echo "rc=$?"
