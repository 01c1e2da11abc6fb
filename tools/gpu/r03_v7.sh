set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="--c5-hosts 0 --text-lines 0 --pcie-steps 0 --timing-steps 0 --steps 12 --warmup 2"
VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py $B --pipeline 1 > gpurun_out/r03_v7_top1.json 2> gpurun_out/r03_v7_top1.log &&
VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py $B --pipeline 3 > gpurun_out/r03_v7_top3.json 2> gpurun_out/r03_v7_top3.log &&
timeout -k 10 400 python -u bench.py $B --pipeline 1 > gpurun_out/r03_v7_base1.json 2> gpurun_out/r03_v7_base1.log
echo "rc=$?"
