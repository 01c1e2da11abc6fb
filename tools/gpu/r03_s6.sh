set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 > gpurun_out/r03_hb6.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 20000 --keys 2000 --reps 2 --no-check >> gpurun_out/r03_hb6.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 20000 --keys 100 --reps 2 --no-check >> gpurun_out/r03_hb6.log 2>&1
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_parity_gpu.py -k histo >> gpurun_out/r03_hb6.log 2>&1
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --c5-hosts 0 --text-lines 0 --pcie-steps 0 --no-cpu-baseline > gpurun_out/r03_b2.json 2> gpurun_out/r03_b2.log
echo done
