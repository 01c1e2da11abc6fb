# C2 one lane per column (VN_C2_LANE variant): batched-replay parity tests, 17M key vs the product, phase cycles
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c2l}
VN_LIB=libveneur_amd_c2l.so timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 &&
VN_LIB=libveneur_amd_c2l.so timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot_base.log 2>&1 &&
VN_LIB=libveneur_amd_c2lp.so timeout -k 10 200 python -u tools/exact_profile.py 4000000 > gpurun_out/${T}_prof.log 2>&1
echo "rc=$?"
