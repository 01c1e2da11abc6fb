set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --rates > gpurun_out/r03_hb7.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --cold-keys 200000 --cold-n 100 --no-check >> gpurun_out/r03_hb7.log 2>&1
timeout -k 10 200 python -u tools/hot_replay_bench.py --n 1000000 --keys 1 --cold-keys 20000 --cold-n 1000 --no-check >> gpurun_out/r03_hb7.log 2>&1
echo done
