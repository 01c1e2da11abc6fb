set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for lib in libveneur_amd.so libveneur_amd_variant.so; do
echo "== $lib"
VN_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py -v --timeout 150 --timeout-method thread 2>&1 | grep -E "PASS|FAIL|Error|centroids|passed|failed" | head -30
done > gpurun_out/r04_a2.log 2>&1
echo "rc=$?"
