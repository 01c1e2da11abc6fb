set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_hot_detect_gpu.py tests/test_split_gpu.py tests/test_import_gpu.py > gpurun_out/r03_h1_tests.log 2>&1 &&
timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --c5-hosts 0 --text-lines 0 --pcie-steps 0 > gpurun_out/r03_h1_bench.json 2> gpurun_out/r03_h1_bench.log
echo "rc=$?"
