set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for b in 268435456; do
timeout -k 10 300 python -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 --c5-batch $b --c5-windows 2 > gpurun_out/r03_c5b_$b.json 2> gpurun_out/r03_c5b_$b.log || exit 1
done
echo "rc=$?"
