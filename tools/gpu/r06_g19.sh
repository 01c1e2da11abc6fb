set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_u
VN_LIB=libveneur_amd_setprof16.so timeout -k 10 200 python -u tools/set_profile.py > gpurun_out/${T}_setprof16.log 2>&1 || exit 11
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 20 --timing-steps 0"
for D in 4 6; do for HQ in 16 32; do
GPU_MAX_HW_QUEUES=$HQ timeout -k 10 400 python -u bench.py $S --pipeline $D > gpurun_out/${T}_sim_8_3_${D}_q${HQ}.json 2> gpurun_out/${T}_sim_8_3_${D}_q${HQ}.log || exit 13
done; done
echo done
