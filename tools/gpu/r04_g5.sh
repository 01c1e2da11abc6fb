set -o pipefail
cd $GRAFT_REPO_ROOT
export HWQ=32
bash tools/gpu/r04_sim.sh s4d2r0 8 "3" --pipeline 2 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s4d3r0 8 "3" --pipeline 3 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s4d3 8 "3" --pipeline 3 &&
bash tools/gpu/r04_sim.sh s4d2 8 "3" --pipeline 2 &&
export GPU_MAX_HW_QUEUES=32 &&
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0 > gpurun_out/r04_g5_n1d2.json 2> gpurun_out/r04_g5_n1d2.log &&
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0 --pipeline 3 > gpurun_out/r04_g5_n1d3.json 2> gpurun_out/r04_g5_n1d3.log
echo "rc=$?"
