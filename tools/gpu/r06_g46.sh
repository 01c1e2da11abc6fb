set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_f4
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
bash tools/gpu/run.sh $T tests smoke bench bench1 prof pmc c5prof hot || exit $?
for D in 3 5 6; do
timeout -k 10 170 python -u bench.py $Q --pipeline $D > gpurun_out/${T}_n1_$D.json 2> gpurun_out/${T}_n1_$D.log || exit 11
done
for s in 2-1 2-0 4-3 4-0 8-3 8-0; do for D in 4 6 7; do
W=${s%-*}; R=${s#*-}
timeout -k 10 170 python -u bench.py $Q --sim-world $W --sim-rank $R --pipeline $D > gpurun_out/${T}_sim_${W}_${R}_$D.json 2> gpurun_out/${T}_sim_${W}_${R}_$D.log || exit 12
done; done
echo done
