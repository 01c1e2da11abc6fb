set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_b1m
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2 3; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 11
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_1m_$k.json 2> gpurun_out/${T}_1m_$k.log || exit 12
done
echo done
