set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u tools/debug_fast.py > gpurun_out/r03_dbg_fast.log 2>&1
VN_LIB=libveneur_amd_variant.so timeout -k 10 120 python -u tools/debug_fast.py 8400 > gpurun_out/r03_dbg_nofast.log 2>&1
echo done
