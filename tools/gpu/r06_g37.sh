set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_bk
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
VN_LIB=libveneur_amd_variant.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_vartests.log 2>&1 || exit 10
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main4_$k.json 2> gpurun_out/${T}_main4_$k.log || exit 11
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_bulk4_$k.json 2> gpurun_out/${T}_bulk4_$k.log || exit 12
VN_LIB=libveneur_amd_bulkasync.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_bulkasync4_$k.json 2> gpurun_out/${T}_bulkasync4_$k.log || exit 13
done
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --pipeline 5 > gpurun_out/${T}_bulk5.json 2> gpurun_out/${T}_bulk5.log || exit 14
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --pipeline 3 > gpurun_out/${T}_bulk3.json 2> gpurun_out/${T}_bulk3.log || exit 15
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 > gpurun_out/${T}_bulk_8_3.json 2> gpurun_out/${T}_bulk_8_3.log || exit 16
timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 > gpurun_out/${T}_main_8_3.json 2> gpurun_out/${T}_main_8_3.log || exit 17
echo done
