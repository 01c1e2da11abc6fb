set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_mk
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 11
VN_LIB=libveneur_amd_re8.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_re8_$k.json 2> gpurun_out/${T}_re8_$k.log || exit 12
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_sideall_$k.json 2> gpurun_out/${T}_sideall_$k.log || exit 13
done
GPU_MAX_HW_QUEUES=32 timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_q32_4.json 2> gpurun_out/${T}_q32_4.log || exit 14
GPU_MAX_HW_QUEUES=32 timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 --pipeline 8 > gpurun_out/${T}_q32_8_3_8.json 2> gpurun_out/${T}_q32_8_3_8.log || exit 15
timeout -k 10 300 python -u bench.py --pipeline 5 > gpurun_out/${T}_full5.json 2> gpurun_out/${T}_full5.log || echo "full5 rc=$?"
echo done
