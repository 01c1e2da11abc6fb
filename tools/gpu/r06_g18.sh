set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_t
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_import_gpu.py tests/test_c3_full_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 10
VN_LIB=libveneur_amd_setprof.so timeout -k 10 200 python -u tools/set_profile.py > gpurun_out/${T}_setprof32.log 2>&1 || exit 11
VN_LIB=libveneur_amd_setprof16.so timeout -k 10 200 python -u tools/set_profile.py > gpurun_out/${T}_setprof16.log 2>&1 || exit 12
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 13
echo done
