set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hot_detect_gpu.py > gpurun_out/r03_h3_tests.log 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_h3 -o h3 --output-format csv -- python3 -u bench.py --steps 1 --warmup 0 --timing-steps 0 --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_h3_prof.json 2> gpurun_out/r03_h3_prof.log
echo "rc=$?"
