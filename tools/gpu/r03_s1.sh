set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parity_gpu.py tests/test_split_gpu.py tests/test_configs_gpu.py tests/test_import_gpu.py > gpurun_out/r03_t1.log 2>&1 ; echo "tests rc=$?" >> gpurun_out/r03_t1.log
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 > gpurun_out/r03_hb1.log 2>&1 && \
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 200000 --keys 64 --reps 2 >> gpurun_out/r03_hb1.log 2>&1 && \
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --fast >> gpurun_out/r03_hb1.log 2>&1
echo done
