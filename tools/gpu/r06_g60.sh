set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_dbg
VN_LIB=libveneur_amd_dbg.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
VN_LIB=libveneur_amd_dbg.so timeout -k 10 200 python -u bench.py $Q > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log || exit 11
for k in 1 2 3; do
timeout -k 10 200 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 12
done
timeout -k 10 200 python -u bench.py $Q --sim-world 2 --sim-rank 1 > gpurun_out/${T}_sim21.json 2> gpurun_out/${T}_sim21.log || exit 13
echo done
