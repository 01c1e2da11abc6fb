set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_sb
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
VN_LIB=libveneur_amd_setprof.so timeout -k 10 300 python -u tools/set_profile.py > gpurun_out/${T}_setprof3.log 2>&1 || exit 11
bash tools/gpu/run.sh $T prof || exit 12
for k in 1 2; do
timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_main_$k.json 2> gpurun_out/${T}_main_$k.log || exit 13
VN_LIB=libveneur_amd_variant.so timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_two_$k.json 2> gpurun_out/${T}_two_$k.log || exit 14
done
timeout -k 10 300 python -u bench.py --c5-only > gpurun_out/${T}_c5.json 2> gpurun_out/${T}_c5.log || exit 15
VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u bench.py --c5-only > gpurun_out/${T}_c5two.json 2> gpurun_out/${T}_c5two.log || exit 16
echo done
