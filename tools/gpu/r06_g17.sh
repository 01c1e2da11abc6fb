set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_s
VN_LIB=libveneur_amd_dbg.so timeout -k 10 600 python -u -m pytest -x -q -s --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_batch_replay_gpu.py tests/test_stream_gpu.py > gpurun_out/${T}_dbg_tests.log 2>&1 || exit 10
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 20 --timing-steps 0"
GPU_MAX_HW_QUEUES=32 VN_LIB=libveneur_amd_dbg.so timeout -k 10 400 python -u bench.py $S --pipeline 4 > gpurun_out/${T}_dbg_sim_8_3_4_q32.json 2> gpurun_out/${T}_dbg_sim_8_3_4_q32.log || exit 11
grep -c VN_CHECK gpurun_out/${T}_dbg_tests.log gpurun_out/${T}_dbg_sim_8_3_4_q32.json gpurun_out/${T}_dbg_sim_8_3_4_q32.log > gpurun_out/${T}_dbg_checks.txt || true
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_import_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 12
VN_LIB=libveneur_amd_setprof.so timeout -k 10 200 python -u tools/set_profile.py > gpurun_out/${T}_setprof_group.log 2>&1 || exit 13
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 14
echo done
