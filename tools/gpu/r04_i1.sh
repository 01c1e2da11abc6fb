set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu/r04_sim.sh ns4 4 "3 0" --no-split &&
bash tools/gpu/r04_sim.sh ns2 2 "1 0" --no-split &&
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 12 --timing-steps 0 --pcie-steps 0 --no-split > gpurun_out/r04_i1_n1ns.json 2> gpurun_out/r04_i1_n1ns.log
echo "rc=$?"
