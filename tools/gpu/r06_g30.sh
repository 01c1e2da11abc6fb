set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_ts tests pmc pmcvar benchq benchqvar benchq benchqvar hot || exit $?
echo done
