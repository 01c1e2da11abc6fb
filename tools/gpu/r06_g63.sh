set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_f9 tests smoke bench bench1 prof pmc c5prof hot || exit $?
echo done
