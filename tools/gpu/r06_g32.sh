set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_cs
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
bash tools/gpu/run.sh $T prof pmc || exit 11
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main4.json 2> gpurun_out/${T}_main4.log || exit 12
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_async4.json 2> gpurun_out/${T}_async4.log || exit 13
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main4b.json 2> gpurun_out/${T}_main4b.log || exit 14
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_async4b.json 2> gpurun_out/${T}_async4b.log || exit 15
echo done
