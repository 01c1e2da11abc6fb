set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_et
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py tests/test_stream_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${T}_vartests.log 2>&1 || exit 10
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 11
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_early_$k.json 2> gpurun_out/${T}_early_$k.log || exit 12
done
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 > gpurun_out/${T}_early_8_3.json 2> gpurun_out/${T}_early_8_3.log || exit 13
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --sim-world 2 --sim-rank 1 > gpurun_out/${T}_early_2_1.json 2> gpurun_out/${T}_early_2_1.log || exit 14
echo done
