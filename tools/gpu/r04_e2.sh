set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12"
timeout -k 10 300 $B > gpurun_out/r04_e2_q4.json 2> gpurun_out/r04_e2_q4.log &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B > gpurun_out/r04_e2_q16.json 2> gpurun_out/r04_e2_q16.log &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --pipeline 3 > gpurun_out/r04_e2_q16d3.json 2> gpurun_out/r04_e2_q16d3.log &&
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 $B --pipeline 3 > gpurun_out/r04_e2_q32d3.json 2> gpurun_out/r04_e2_q32d3.log
echo "rc=$?"
