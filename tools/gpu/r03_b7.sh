set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --rates > gpurun_out/r03_b7.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --no-check --reps 2 >> gpurun_out/r03_b7.log 2>&1 &&
for v in prof prof_rolled; do echo "== $v"; VN_LIB=libveneur_amd_$v.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 || exit 1; done >> gpurun_out/r03_b7.log 2>&1
echo "rc=$?"
