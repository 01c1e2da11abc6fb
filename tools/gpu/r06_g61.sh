set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_d6
timeout -k 10 300 python -u bench.py --pipeline 6 > gpurun_out/${T}_full6.json 2> gpurun_out/${T}_full6.log || echo "full6 rc=$?"
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_full5.json 2> gpurun_out/${T}_full5.log || exit 11
echo done
