set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_e
timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 3 > gpurun_out/${T}_prod.log 2>&1; rc=$?; echo "prod rc=$rc"
if [ $rc -ne 0 ]; then exit 11; fi
timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 2 > gpurun_out/${T}_prod2.log 2>&1; rc=$?; echo "prod2 rc=$rc"
if [ $rc -ne 0 ]; then exit 12; fi
VN_LIB=libveneur_amd_check.so timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 3 > gpurun_out/${T}_check.log 2>&1; rc=$?; echo "check rc=$rc"
echo done
