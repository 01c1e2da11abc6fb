set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_import_gpu.py tests/test_edges_gpu.py tests/test_http_import.py > gpurun_out/r03_s3_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 > gpurun_out/r03_s3_bench.json 2> gpurun_out/r03_s3_bench.log &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_s3 -o c5 --output-format csv -- python3 -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 > gpurun_out/r03_s3_prof.json 2> gpurun_out/r03_s3_prof.log
echo "rc=$?"
