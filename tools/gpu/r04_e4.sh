set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
B="bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 6 --timing-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_e4_r0 -o r0 -- python3 $B --reserved-cus 0 > gpurun_out/r04_e4_r0.json 2> gpurun_out/r04_e4_r0.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r04_e4_r16 -o r16 -- python3 $B --reserved-cus 16 > gpurun_out/r04_e4_r16.json 2> gpurun_out/r04_e4_r16.log
echo "rc=$?"
