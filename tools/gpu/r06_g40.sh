set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_fd
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || exit 10
for D in 4 5 6; do
timeout -k 10 170 python -u bench.py $Q --pipeline $D > gpurun_out/${T}_n1_$D.json 2> gpurun_out/${T}_n1_$D.log || exit 11
done
for s in 2-1 2-0 4-3 4-0 8-3 8-0; do for D in 4 6; do
W=${s%-*}; R=${s#*-}
timeout -k 10 170 python -u bench.py $Q --sim-world $W --sim-rank $R --pipeline $D > gpurun_out/${T}_sim_${W}_${R}_$D.json 2> gpurun_out/${T}_sim_${W}_${R}_$D.log || exit 12
done; done
timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 --pipeline 5 > gpurun_out/${T}_sim_8_3_5.json 2> gpurun_out/${T}_sim_8_3_5.log || exit 13
timeout -k 10 170 python -u bench.py $Q --sim-world 8 --sim-rank 3 --pipeline 7 > gpurun_out/${T}_sim_8_3_7.json 2> gpurun_out/${T}_sim_8_3_7.log || exit 14
echo done
