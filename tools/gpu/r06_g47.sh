set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_f5 bench || exit $?
echo done
