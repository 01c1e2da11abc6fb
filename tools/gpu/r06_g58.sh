set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_t5
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 11
VN_LIB=libveneur_amd_lm128k.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_lm128k_$k.json 2> gpurun_out/${T}_lm128k_$k.log || exit 12
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_bm512k_$k.json 2> gpurun_out/${T}_bm512k_$k.log || exit 13
done
echo done
