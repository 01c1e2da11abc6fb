set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_s2 -o c5 --output-format csv -- python3 -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 > gpurun_out/r03_s2.json 2> gpurun_out/r03_s2.log
echo "rc=$?"
