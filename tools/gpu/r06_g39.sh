set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_fm
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main4.json 2> gpurun_out/${T}_main4.log || exit 11
for D in 4 5 6; do
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --pipeline $D > gpurun_out/${T}_fm$D.json 2> gpurun_out/${T}_fm$D.log || exit 12
done
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 --pipeline 6 > gpurun_out/${T}_fm_8_3_6.json 2> gpurun_out/${T}_fm_8_3_6.log || exit 13
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 > gpurun_out/${T}_fm_8_3_4.json 2> gpurun_out/${T}_fm_8_3_4.log || exit 14
echo done
