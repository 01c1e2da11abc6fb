set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_k
timeout -k 10 300 python -u tools/scalar_bench.py --steps 10 --check > gpurun_out/${T}_scalar.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_scalar_prof -o scalar -- python -u tools/scalar_bench.py --steps 5 > gpurun_out/${T}_scalar_prof.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_edges_gpu.py tests/test_stream_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 12
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batch_replay_gpu.py > gpurun_out/${T}_rep_tests.log 2>&1 || exit 13
VN_LIB=libveneur_amd_prof.so timeout -k 10 200 python -u tools/exact_profile.py 4000000 > gpurun_out/${T}_prof4M_rep.log 2>&1 || exit 14
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot17M_rep.log 2>&1 || exit 15
echo done
