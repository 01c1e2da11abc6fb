set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_f
for v in vA vB vC; do
  VN_LIB=libveneur_amd_$v.so timeout -k 10 300 python -u tools/probe/repro_batch3_calls.py 3 > gpurun_out/${T}_$v.log 2>&1; rc=$?; echo "$v rc=$rc"
  if [ $rc -ne 0 ]; then exit 11; fi
done
echo done
