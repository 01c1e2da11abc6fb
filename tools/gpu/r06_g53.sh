set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_mem
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
timeout -k 10 300 python -u bench.py --pipeline 6 > gpurun_out/${T}_full6.json 2> gpurun_out/${T}_full6.log || echo "full6 rc=$?"
timeout -k 10 300 python -u bench.py --pipeline 5 > gpurun_out/${T}_full5.json 2> gpurun_out/${T}_full5.log || echo "full5 rc=$?"
timeout -k 10 300 python -u bench.py > gpurun_out/${T}_full4.json 2> gpurun_out/${T}_full4.log || exit 13
echo done
