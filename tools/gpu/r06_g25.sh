set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_aa
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_worker_rotation_gpu.py tests/test_split_gpu.py tests/test_pipeline_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 10
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for D in 3 4; do
echo "bench D=$D $(date +%T)" >> gpurun_out/${T}_progress.txt
timeout -k 10 170 python -u bench.py $Q --pipeline $D > gpurun_out/${T}_bench_$D.json 2> gpurun_out/${T}_bench_$D.log || exit 11
done
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 20 --timing-steps 0"
for D in 4 5 6; do
echo "sim D=$D $(date +%T)" >> gpurun_out/${T}_progress.txt
timeout -k 10 170 python -u bench.py $S --pipeline $D > gpurun_out/${T}_sim_8_3_$D.json 2> gpurun_out/${T}_sim_8_3_$D.log || exit 12
done
echo done
