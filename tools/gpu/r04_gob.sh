# gob decode change: import tests, then the C5 leg's phases
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-gob}
VN_LIB=${LIB:-libveneur_amd.so} timeout -k 10 400 python -u -m pytest tests/test_import_gpu.py tests/test_import_sharded_gpu.py tests/test_edges_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 &&
VN_LIB=${LIB:-libveneur_amd.so} timeout -k 10 300 python -u tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/${T}_c5.log 2>&1
echo "rc=$?"
