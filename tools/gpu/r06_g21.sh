set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_w
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2; do for V in prod R0 C0; do
L=libveneur_amd.so; [ $V != prod ] && L=libveneur_amd_$V.so
echo "run $k $V $(date +%T)" >> gpurun_out/${T}_progress.txt
VN_LIB=$L timeout -k 10 170 python -u bench.py $Q > gpurun_out/${T}_bench_${V}_${k}.json 2> gpurun_out/${T}_bench_${V}_${k}.log || { echo "FAILED $V $k rc=$?" >> gpurun_out/${T}_progress.txt; exit 13; }
done; done
echo done
