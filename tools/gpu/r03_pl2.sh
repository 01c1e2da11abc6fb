set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
B="--c5-hosts 0 --text-lines 0 --pcie-steps 0 --timing-steps 0"
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 $B --pipeline 1 > gpurun_out/r03_pl2_base1.json 2> gpurun_out/r03_pl2_base1.log &&
VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 $B --pipeline 1 > gpurun_out/r03_pl2_ex1.json 2> gpurun_out/r03_pl2_ex1.log &&
VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 $B --pipeline 2 > gpurun_out/r03_pl2_ex2.json 2> gpurun_out/r03_pl2_ex2.log
echo "rc=$?"
