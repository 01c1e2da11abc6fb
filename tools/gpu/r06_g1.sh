set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_a
true
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
VN_LIB=libveneur_amd_check.so timeout -k 10 600 $P tests/test_batch_replay_gpu.py > gpurun_out/${T}_check.log 2>&1 || exit 11
VN_LIB=libveneur_amd_nrcheck.so timeout -k 10 300 $P tests/test_batch_replay_gpu.py -k "whole_digest_bit_exact and 1" -s > gpurun_out/${T}_nrcheck.log 2>&1; rc=$?
echo "nrcheck rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 12; fi
timeout -k 10 600 $P tests/test_worker_rotation_gpu.py tests/test_sink.py > gpurun_out/${T}_rot.log 2>&1 || exit 13
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 14
VN_LIB=libveneur_amd_noexcl.so timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq_noexcl.json 2> gpurun_out/${T}_benchq_noexcl.log || exit 15
timeout -k 10 400 python -u bench.py $Q --pipeline 4 > gpurun_out/${T}_benchq4.json 2> gpurun_out/${T}_benchq4.log || exit 16
echo done
