set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_f2 tests smoke bench bench1 prof pmc c5prof hot sim-2-0-4 sim-2-1-4 sim-8-0-4 sim-8-3-4 || exit $?
echo done
