# C5: the global engine's import run size (drain slices) A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c5b}
timeout -k 10 500 python -u tools/c5_check.py 1000,10000,2000,67108864 1000,10000,2000,268435456 1000,10000,2000,805306368 > gpurun_out/${T}.log 2>&1
echo "rc=$?"
