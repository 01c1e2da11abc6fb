# parity of the replay after a codegen change, the 17M key, PMC traffic, then the default bench with 3 engines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-scr}
timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py tests/test_parity_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot.log 2>&1 &&
bash tools/gpu/r04_pmc.sh ${T}_pmc &&
timeout -k 10 500 python bench.py --pipeline 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log
echo "rc=$?"
