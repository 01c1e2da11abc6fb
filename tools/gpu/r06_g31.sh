set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_hw
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_async4.json 2> gpurun_out/${T}_async4.log || exit 11
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_waits4.json 2> gpurun_out/${T}_waits4.log || exit 12
timeout -k 10 170 python -u bench.py $Q --pipeline 3 > gpurun_out/${T}_async3.json 2> gpurun_out/${T}_async3.log || exit 13
timeout -k 10 170 python -u bench.py $Q --pipeline 6 > gpurun_out/${T}_async6.json 2> gpurun_out/${T}_async6.log || exit 14
timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 > gpurun_out/${T}_async_8_3.json 2> gpurun_out/${T}_async_8_3.log || exit 15
timeout -k 10 170 python -u bench.py $Q --no-stagger > gpurun_out/${T}_async4_nostagger.json 2> gpurun_out/${T}_async4_nostagger.log || exit 16
echo done
