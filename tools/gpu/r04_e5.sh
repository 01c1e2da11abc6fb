set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
B="python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12"
timeout -k 10 300 $B --reserved-cus 0 > gpurun_out/r04_e5_r0.json 2> gpurun_out/r04_e5_r0.log &&
timeout -k 10 300 $B --reserved-cus 16 > gpurun_out/r04_e5_r16.json 2> gpurun_out/r04_e5_r16.log &&
timeout -k 10 300 $B --reserved-cus 0 --no-stagger > gpurun_out/r04_e5_ns.json 2> gpurun_out/r04_e5_ns.log &&
timeout -k 10 300 $B --reserved-cus 0 --pipeline 3 > gpurun_out/r04_e5_d3.json 2> gpurun_out/r04_e5_d3.log
echo "rc=$?"
