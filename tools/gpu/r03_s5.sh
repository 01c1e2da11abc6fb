set -o pipefail
cd $GRAFT_REPO_ROOT
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 1000000 > gpurun_out/r03_exact_prof.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 >> gpurun_out/r03_exact_prof.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 200000 --keys 64 --reps 2 >> gpurun_out/r03_exact_prof.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_parity_gpu.py -k histo > gpurun_out/r03_t5.log 2>&1; echo "rc=$?" >> gpurun_out/r03_t5.log
VN_LIB=libveneur_amd_variant.so timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_parity_gpu.py -k "c4_hot_key_sizes_exact or exact_replay" > gpurun_out/r03_t5_nopred.log 2>&1; echo "rc=$?" >> gpurun_out/r03_t5_nopred.log
echo done
