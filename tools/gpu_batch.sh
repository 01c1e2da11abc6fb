# one gpurun call: replay / import parity tests, the exact-replay phase profile, a serialized N=1 kernel trace
set -e
cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/t_all.log 2>&1
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python tools/exact_profile.py > gpurun_out/exact_prof.txt 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl6 -o tl -- python bench.py --steps 1 --warmup 1 --timing-steps 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/tl6.log 2>&1
