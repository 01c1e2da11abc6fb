set -o pipefail
cd $GRAFT_REPO_ROOT
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 1000000 > gpurun_out/r03_exact_prof.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 >> gpurun_out/r03_exact_prof.log 2>&1
echo done
