set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_c4prof -o c4 --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --timing-steps 0 --no-cpu-baseline --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_c4prof.json 2> gpurun_out/r03_c4prof.log
echo done
