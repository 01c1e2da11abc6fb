set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_import_gpu.py tests/test_edges_gpu.py tests/test_http_import.py tests/test_configs_gpu.py tests/test_worker.py > gpurun_out/r03_v11_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --keys 10000 --samples 10000000 --steps 1 --warmup 0 --timing-steps 0 --pcie-steps 0 --text-lines 0 --pipeline 1 > gpurun_out/r03_v11_c5.json 2> gpurun_out/r03_v11_c5.log
echo "rc=$?"
