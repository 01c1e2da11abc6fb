set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
H="python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 --no-check"
timeout -k 10 300 $H --engines 2 > gpurun_out/r04_g2_e2.log 2>&1 &&
timeout -k 10 300 $H --engines 3 > gpurun_out/r04_g2_e3.log 2>&1 &&
timeout -k 10 300 $H --engines 2 --cold-keys 1000000 --cold-n 400 > gpurun_out/r04_g2_e2cold.log 2>&1
echo "rc=$?"
