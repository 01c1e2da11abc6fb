set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/r04_g6 -o d3 -- python3 bench.py --sim-world 8 --sim-rank 3 --steps 6 --warmup 1 --c5-hosts 0 --text-lines 0 --timing-steps 0 --pcie-steps 0 --pipeline 3 --reserved-cus 0 > gpurun_out/r04_g6.json 2> gpurun_out/r04_g6.log
echo "rc=$?"
