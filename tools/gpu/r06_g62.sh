set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_cpw
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py tests/test_stream_gpu.py -x -q --timeout 250 --timeout-method thread > gpurun_out/${T}_tests4.log 2>&1 || exit 11
bash tools/gpu/run.sh $T prof || exit 12
VN_LIB=libveneur_amd_cpw1.so bash tools/gpu/run.sh ${T}1 prof || exit 13
VN_LIB=libveneur_amd_variant.so bash tools/gpu/run.sh ${T}4 prof || exit 14
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 15
VN_LIB=libveneur_amd_cpw1.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_k1_$k.json 2> gpurun_out/${T}_k1_$k.log || exit 16
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_k4_$k.json 2> gpurun_out/${T}_k4_$k.log || exit 17
done
echo done
