set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
B="python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0"
timeout -k 10 300 $B --pipeline 2 --reserved-cus 16 > gpurun_out/r04_e6_d2r16.json 2> gpurun_out/r04_e6_d2r16.log &&
timeout -k 10 300 $B --pipeline 3 --reserved-cus 24 > gpurun_out/r04_e6_d3r24.json 2> gpurun_out/r04_e6_d3r24.log &&
timeout -k 10 300 $B --pipeline 3 --reserved-cus 0 > gpurun_out/r04_e6_d3r0.json 2> gpurun_out/r04_e6_d3r0.log &&
timeout -k 10 300 $B --pipeline 4 --reserved-cus 32 > gpurun_out/r04_e6_d4r32.json 2> gpurun_out/r04_e6_d4r32.log &&
timeout -k 10 300 $B --pipeline 2 --reserved-cus 0 > gpurun_out/r04_e6_d2r0.json 2> gpurun_out/r04_e6_d2r0.log
echo "rc=$?"
