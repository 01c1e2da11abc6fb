set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_f8 tests smoke bench bench1 prof pmc c5prof hot sim-2-1-7 sim-2-0-7 sim-4-3-7 sim-4-0-7 sim-8-3-7 sim-8-0-7 || exit $?
echo done
