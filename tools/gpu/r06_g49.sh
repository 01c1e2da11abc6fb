set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_ls
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 11
VN_LIB=libveneur_amd_lr16k.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_64k_$k.json 2> gpurun_out/${T}_64k_$k.log || exit 12
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_128k_$k.json 2> gpurun_out/${T}_128k_$k.log || exit 13
done

VN_LIB=libveneur_amd_lr16k.so timeout -k 10 300 python -u bench.py --c5-only > gpurun_out/r06_ls_c5_64k.json 2> gpurun_out/r06_ls_c5_64k.log || exit 14
echo done
