set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 400 --timeout-method thread > gpurun_out/r04_b3_tests.log 2>&1 &&
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 > gpurun_out/r04_b3_prof.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/r04_b3_hot.log 2>&1
echo "rc=$?"
