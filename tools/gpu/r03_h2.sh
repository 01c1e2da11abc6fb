set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_h2_bench.json 2> gpurun_out/r03_h2_bench.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_h2 -o h2 --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --timing-steps 0 --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_h2_prof.json 2> gpurun_out/r03_h2_prof.log
echo "rc=$?"
