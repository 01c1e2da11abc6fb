set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests > gpurun_out/r03_v6_tests.log 2>&1 || { echo "tests failed"; exit 1; }
B="--c5-hosts 0 --text-lines 0 --pcie-steps 0 --timing-steps 0 --steps 12 --warmup 2"
timeout -k 10 400 python -u bench.py $B --pipeline 1 > gpurun_out/r03_v6_base1.json 2> gpurun_out/r03_v6_base1.log &&
timeout -k 10 400 python -u bench.py $B --pipeline 2 > gpurun_out/r03_v6_base2.json 2> gpurun_out/r03_v6_base2.log &&
VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py $B --pipeline 2 > gpurun_out/r03_v6_top2.json 2> gpurun_out/r03_v6_top2.log &&
timeout -k 10 300 python -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 --pipeline 1 > gpurun_out/r03_v6_c5.json 2> gpurun_out/r03_v6_c5.log
echo "rc=$?"
