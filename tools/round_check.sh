# One gpurun call at a milestone: the GPU tests, smoke, the default bench line, and the rocprofv3
# kernel statistics of a short bench run (outputs under gpurun_out/, TAG names them).
set -e
TAG=${1:-rXX}
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 250 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --pcie-steps 0 > gpurun_out/${TAG}_prof.log 2>&1
