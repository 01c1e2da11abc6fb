set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_batch_replay_gpu.py tests/test_parity_gpu.py tests/test_import_gpu.py tests/test_split_gpu.py -x -v --timeout 150 --timeout-method thread -k "batch or four_wave or hot_key_sizes_exact or import or split_slot" > gpurun_out/r04_a7_tests.log 2>&1 &&
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 4000000 --keys 1 --rates > gpurun_out/r04_a7_hot.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 >> gpurun_out/r04_a7_hot.log 2>&1
echo "rc=$?"
