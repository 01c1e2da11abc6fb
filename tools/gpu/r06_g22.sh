set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_x
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_batch_replay_gpu.py tests/test_c3_full_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 10
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2 3; do
echo "bench $k $(date +%T)" >> gpurun_out/${T}_progress.txt
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_bench_${k}.json 2> gpurun_out/${T}_bench_${k}.log || { echo "FAILED bench $k rc=$?" >> gpurun_out/${T}_progress.txt; exit 13; }
done
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 20 --timing-steps 0"
for D in 4 6; do
echo "sim $D $(date +%T)" >> gpurun_out/${T}_progress.txt
timeout -k 10 170 python -u bench.py $S --pipeline $D > gpurun_out/${T}_sim_8_3_${D}.json 2> gpurun_out/${T}_sim_8_3_${D}.log || { echo "FAILED sim $D rc=$?" >> gpurun_out/${T}_progress.txt; exit 14; }
done
echo done
