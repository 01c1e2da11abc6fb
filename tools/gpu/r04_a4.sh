set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/debug_prefix.py debug/debug_rising.npz 25362 > gpurun_out/r04_a4.log 2>&1 &&
timeout -k 10 120 python -u tools/debug_prefix.py debug/debug_rising.npz 25361 >> gpurun_out/r04_a4.log 2>&1
echo "rc=$?"
