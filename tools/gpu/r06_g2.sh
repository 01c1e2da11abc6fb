set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_b
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $P tests/test_batch_replay_gpu.py tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_stream_gpu.py tests/test_worker_rotation_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 11
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 14
VN_LIB=libveneur_amd_nopo.so timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq_nopo.json 2> gpurun_out/${T}_benchq_nopo.log || exit 15
# the round-5 all-sites NR build, once, on the test that gave a wrong digest then
VN_LIB=libveneur_amd_nr.so timeout -k 10 300 $P tests/test_batch_replay_gpu.py -k "whole_digest_bit_exact and 1" > gpurun_out/${T}_nr.log 2>&1; rc=$?
echo "nr rc=$rc"
timeout -k 10 300 python -u bench.py --c5-only > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.log || exit 16
echo done
