set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --steps 5 --warmup 1 --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_b1.json 2> gpurun_out/r03_b1.log
echo done
