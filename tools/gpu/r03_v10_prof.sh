set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_v10_prof -o c4 --output-format csv -- python3 -u bench.py --steps 1 --warmup 1 --timing-steps 1 --c5-hosts 0 --no-cpu-baseline --pcie-steps 0 --text-lines 0 --pipeline 1 > gpurun_out/r03_v10_prof.json 2> gpurun_out/r03_v10_prof.log
echo "rc=$?"
