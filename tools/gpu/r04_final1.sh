set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r04_final1_bench.json 2> gpurun_out/r04_final1_bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_final1_prof -o bench -- python3 bench.py --steps 6 --no-cpu-baseline --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r04_final1_prof.json 2> gpurun_out/r04_final1_prof.log
echo "rc=$?"
