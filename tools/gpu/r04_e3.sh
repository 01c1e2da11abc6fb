set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12"
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B > gpurun_out/r04_e3_r16.json 2> gpurun_out/r04_e3_r16.log &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --reserved-cus 0 > gpurun_out/r04_e3_r0.json 2> gpurun_out/r04_e3_r0.log &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --pipeline 3 > gpurun_out/r04_e3_d3.json 2> gpurun_out/r04_e3_d3.log &&
GPU_MAX_HW_QUEUES=16 timeout -k 10 300 $B --pipeline 1 > gpurun_out/r04_e3_d1.json 2> gpurun_out/r04_e3_d1.log
echo "rc=$?"
