set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_f6
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
bash tools/gpu/run.sh $T tests smoke bench bench1 prof pmc c5prof hot sim-2-1-7 sim-2-0-7 sim-4-3-7 sim-4-0-7 sim-8-3-7 sim-8-0-7 || exit $?
echo done
