set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_v
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_import_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 10
VN_LIB=libveneur_amd_setprof.so timeout -k 10 200 python -u tools/set_profile.py > gpurun_out/${T}_setprof.log 2>&1 || exit 11
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 12
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 20 --timing-steps 0"
for D in 4 6; do
timeout -k 10 400 python -u bench.py $S --pipeline $D > gpurun_out/${T}_sim_8_3_${D}.json 2> gpurun_out/${T}_sim_8_3_${D}.log || exit 13
done
echo done
