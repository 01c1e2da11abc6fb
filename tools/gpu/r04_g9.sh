set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r04_sim.sh s6d2 8 "3" --pipeline 2 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s6d3 8 "3" --pipeline 3 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s6d4 8 "3" --pipeline 4 --reserved-cus 0 &&
bash tools/gpu/r04_sim.sh s6d3r 8 "3" --pipeline 3 --reserved-cus 24 &&
export GPU_MAX_HW_QUEUES=16 &&
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0 --pipeline 3 > gpurun_out/r04_g9_n1d3.json 2> gpurun_out/r04_g9_n1d3.log
echo "rc=$?"
