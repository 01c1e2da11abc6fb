set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_v9_smoke.log 2>&1 &&
timeout -k 10 900 python -u bench.py > gpurun_out/r03_v9_bench.json 2> gpurun_out/r03_v9_bench.log
echo "bench rc=$?"
