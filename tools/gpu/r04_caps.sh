# per-class record caps: boundary tests, then C4 at three and four engines in turn
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-caps}
A="--steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u -m pytest tests/test_edges_gpu.py tests/test_import_gpu.py tests/test_intake_gpu.py tests/test_abi.py tests/test_batch_replay_gpu.py tests/test_parity_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 300 python bench.py $A > gpurun_out/${T}_d3.json 2> gpurun_out/${T}_d3.log &&
timeout -k 10 300 python bench.py $A --pipeline 4 > gpurun_out/${T}_d4.json 2> gpurun_out/${T}_d4.log
echo "rc=$?"
