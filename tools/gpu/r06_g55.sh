set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_simfull
timeout -k 10 400 python -u bench.py --sim-world 2 --sim-rank 1 > gpurun_out/${T}_2_1.json 2> gpurun_out/${T}_2_1.log || echo "2_1 rc=$?"
timeout -k 10 400 python -u bench.py --sim-world 2 --sim-rank 0 > gpurun_out/${T}_2_0.json 2> gpurun_out/${T}_2_0.log || echo "2_0 rc=$?"
echo done
