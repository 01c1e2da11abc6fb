set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_c5b
for B in 67108864 134217728 268435456; do
timeout -k 10 300 python -u bench.py --c5-only --c5-batch $B > gpurun_out/${T}_$B.json 2> gpurun_out/${T}_$B.log || echo "c5 $B rc=$?"
done
echo done
