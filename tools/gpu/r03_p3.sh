set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --rates > gpurun_out/r03_p3.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 4000000 --keys 1 --rates >> gpurun_out/r03_p3.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --no-check --reps 2 >> gpurun_out/r03_p3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_stream_gpu.py tests/test_exact_gpu.py >> gpurun_out/r03_p3.log 2>&1
echo "rc=$?"
