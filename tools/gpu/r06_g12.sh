set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_m
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batch_replay_gpu.py > gpurun_out/${T}_rep_tests.log 2>&1 || exit 10
VN_LIB=libveneur_amd_prof.so timeout -k 10 200 python -u tools/exact_profile.py 4000000 > gpurun_out/${T}_prof4M_rep.log 2>&1 || exit 11
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot17M_rep.log 2>&1 || exit 12
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
VN_LIB=libveneur_amd_rep.so timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq_rep.json 2> gpurun_out/${T}_benchq_rep.log || exit 13
for D in 4 6; do
VN_LIB=libveneur_amd_prof.so timeout -k 10 400 python -u bench.py $Q --worker-windows 0 --sim-world 8 --sim-rank 3 --pipeline $D > gpurun_out/${T}_sim_8_3_${D}.json 2> gpurun_out/${T}_sim_8_3_${D}.log || exit 14
done
echo done
