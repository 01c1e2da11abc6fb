set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/r04_b2_tests.log 2>&1 &&
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 > gpurun_out/r04_b2_prof.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/r04_b2_hot.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_pipeline_gpu.py tests/test_import_sharded_gpu.py tests/test_configs_gpu.py -k "pipeline or sharded or c5" -x -v --timeout 150 --timeout-method thread > gpurun_out/r04_b2_pipe.log 2>&1 &&
timeout -k 10 400 python -u -m pytest tests/test_c3_full_gpu.py -x -v --timeout 350 --timeout-method thread > gpurun_out/r04_b2_c3.log 2>&1
echo "rc=$?"
