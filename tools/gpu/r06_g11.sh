set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_l
timeout -k 10 300 python -u tools/scalar_bench.py --steps 10 --check > gpurun_out/${T}_scalar.log 2>&1 || exit 10
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_scalar_prof -o scalar -- python -u tools/scalar_bench.py --steps 5 > gpurun_out/${T}_scalar_prof.log 2>&1 || exit 11
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_parity_gpu.py tests/test_edges_gpu.py tests/test_stream_gpu.py > gpurun_out/${T}_tests.log 2>&1 || exit 12
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 400 python -u bench.py $Q > gpurun_out/${T}_benchq.json 2> gpurun_out/${T}_benchq.log || exit 13
echo done
