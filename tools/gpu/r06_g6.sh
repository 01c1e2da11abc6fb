set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_g
P="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 3 > gpurun_out/${T}_calls.log 2>&1 || exit 10
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 3 > gpurun_out/${T}_rep_calls.log 2>&1 || exit 11
VN_LIB=libveneur_amd_rep.so timeout -k 10 300 $P tests/test_batch_replay_gpu.py > gpurun_out/${T}_rep_batch.log 2>&1 || exit 12
VN_LIB=libveneur_amd_nr.so timeout -k 10 300 $P tests/test_batch_replay_gpu.py > gpurun_out/${T}_nr.log 2>&1 || exit 13
timeout -k 10 900 $P tests -m gpu > gpurun_out/${T}_tests.log 2>&1 || exit 14
echo done
