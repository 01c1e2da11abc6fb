# kernel trace of the default bench (three engines in turn), short legs off
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
T=${1:-tr3}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T} -o run -- python bench.py --steps 10 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.log
echo done
