set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --steps 8 --warmup 2 --c5-hosts 0 --text-lines 0 --pcie-steps 0 --pipeline 2 > gpurun_out/r03_pl1_d2.json 2> gpurun_out/r03_pl1_d2.log &&
timeout -k 10 500 python -u bench.py --steps 9 --warmup 3 --c5-hosts 0 --text-lines 0 --pcie-steps 0 --pipeline 3 > gpurun_out/r03_pl1_d3.json 2> gpurun_out/r03_pl1_d3.log
echo "rc=$?"
