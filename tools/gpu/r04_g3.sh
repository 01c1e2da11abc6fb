set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
H="python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 --no-check"
timeout -k 10 300 $H --engines 2 --cold-keys 1000000 --cold-n 400 --reserved-cus 16 > gpurun_out/r04_g3_e2cold_r16.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 400 --keys 1 --rates --reps 2 --no-check --engines 2 --cold-keys 1000000 --cold-n 400 > gpurun_out/r04_g3_coldonly.log 2>&1 &&
timeout -k 10 300 $H --engines 3 --cold-keys 1000000 --cold-n 400 --reserved-cus 24 > gpurun_out/r04_g3_e3cold_r24.log 2>&1
echo "rc=$?"
