set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_ab
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for k in 1 2; do for D in 3 4 5; do
echo "bench D=$D k=$k $(date +%T)" >> gpurun_out/${T}_progress.txt
timeout -k 10 170 python -u bench.py $Q --pipeline $D > gpurun_out/${T}_bench_${D}_$k.json 2> gpurun_out/${T}_bench_${D}_$k.log || exit 11
done; done
echo done
