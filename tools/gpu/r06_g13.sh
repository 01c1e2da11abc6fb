set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_n
timeout -k 10 300 python -u tools/scalar_bench.py --steps 10 --check > gpurun_out/${T}_scalar.log 2>&1 || exit 10
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_batch_replay_gpu.py tests/test_parity_gpu.py tests/test_edges_gpu.py tests/test_stream_gpu.py tests/test_c3_full_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 11
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_scalar_prof -o scalar -- python -u tools/scalar_bench.py --steps 5 > gpurun_out/${T}_scalar_prof.log 2>&1 || exit 12
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}_hot17M.log 2>&1 || exit 13
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 14
S="$Q --worker-windows 0 --sim-world 8 --sim-rank 3 --steps 12"
GPU_MAX_HW_QUEUES=32 timeout -k 10 400 python -u bench.py $S --pipeline 6 > gpurun_out/${T}_sim_8_3_6_q32.json 2> gpurun_out/${T}_sim_8_3_6_q32.log || exit 15
for D in 4 6; do
VN_LIB=libveneur_amd_nomask.so timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_trace_${D} -o tr -- python -u bench.py $S --pipeline $D --timing-steps 0 > gpurun_out/${T}_trace_${D}.json 2> gpurun_out/${T}_trace_${D}.log || exit 16
done
echo done
