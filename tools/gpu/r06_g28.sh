set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_f2 sim-4-0-4 sim-4-3-4 benchq || exit $?
echo done
