set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py > gpurun_out/r04_c1_bench.json 2> gpurun_out/r04_c1_bench.log
echo "rc=$?"
