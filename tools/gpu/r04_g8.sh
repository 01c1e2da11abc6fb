set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04_g8_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 --engines 2 --cold-keys 1000000 --cold-n 400 > gpurun_out/r04_g8_hot.log 2>&1 &&
bash tools/gpu/r04_sim.sh s5d2 8 "3" --pipeline 2 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s5d3 8 "3" --pipeline 3 --reserved-cus 0 &&
export GPU_MAX_HW_QUEUES=16 &&
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0 > gpurun_out/r04_g8_n1d2.json 2> gpurun_out/r04_g8_n1d2.log
echo "rc=$?"
