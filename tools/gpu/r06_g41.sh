set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_fd
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for s in 2-1 2-0 4-3 4-0 8-3 8-0; do for D in 7 8; do
W=${s%-*}; R=${s#*-}
timeout -k 10 170 python -u bench.py $Q --sim-world $W --sim-rank $R --pipeline $D > gpurun_out/${T}_sim_${W}_${R}_$D.json 2> gpurun_out/${T}_sim_${W}_${R}_$D.log || echo "sim $W $R $D rc=$?"
done; done
echo done
