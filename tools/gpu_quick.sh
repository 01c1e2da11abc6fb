# one gpurun call while iterating: the GPU suite, a short bench line (kernel timings included)
# and the exact-replay phase profile (outputs under gpurun_out/, TAG names them)
set -e
TAG=${1:-q}
cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${TAG}_b.json 2> gpurun_out/${TAG}_b.log
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python tools/exact_profile.py > gpurun_out/${TAG}_exact_prof.txt 2>&1
