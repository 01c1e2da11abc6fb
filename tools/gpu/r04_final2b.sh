# round-4 final check, part 2: the default bench line, then a rocprofv3 kernel summary of a short run
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r04_final2}
timeout -k 10 700 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log &&
cd /tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o bench -- python3 bench.py --steps 6 --no-cpu-baseline --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/${T}_prof.json 2> gpurun_out/${T}_prof.log
echo "rc=$?"
