set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/r04_c5a_plain.log 2>&1 &&
VN_LONG_REPLAY=4096 timeout -k 10 300 python -u tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/r04_c5a_lr4k.log 2>&1 &&
VN_LONG_REPLAY=2048 timeout -k 10 300 python -u tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/r04_c5a_lr2k.log 2>&1 &&
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/r04_c5a_prof -o c5 -- python3 tools/c5_check.py 1000,10000,2000,67108864 > gpurun_out/r04_c5a_prof.log 2>&1
echo "rc=$?"
