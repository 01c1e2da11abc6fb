set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_ch
H="tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2"
timeout -k 10 200 python -u $H > gpurun_out/${T}_main.log 2>&1 || exit 10
for n in REP3 REP6 C2G1 C2G3; do
VN_LIB=libveneur_amd_$n.so timeout -k 10 200 python -u $H > gpurun_out/${T}_$n.log 2>&1 || echo "$n rc=$?"
done
timeout -k 10 200 python -u $H > gpurun_out/${T}_main2.log 2>&1 || exit 11
echo done
