set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_d
timeout -k 10 300 python -u tools/probe/repro_batch3.py 3 > gpurun_out/${T}_prod.log 2>&1; rc=$?; echo "prod rc=$rc"
if [ $rc -ne 0 ]; then exit 11; fi
VN_LIB=libveneur_amd_check.so timeout -k 10 300 python -u tools/probe/repro_batch3.py 3 > gpurun_out/${T}_check.log 2>&1; rc=$?; echo "check rc=$rc"
echo done
