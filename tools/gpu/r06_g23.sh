set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu/run.sh r06_y tests smoke bench bench1 || exit $?
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0"
for D in 4 5; do
echo "[r06_g23] D=$D q32 $(date +%T)"
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python -u bench.py $Q --pipeline $D > gpurun_out/r06_y_benchq${D}_q32.json 2> gpurun_out/r06_y_benchq${D}_q32.log || exit 15
done
echo "[r06_g23] D=3 q32 $(date +%T)"
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python -u bench.py $Q > gpurun_out/r06_y_benchq3_q32.json 2> gpurun_out/r06_y_benchq3_q32.log || exit 16
bash tools/gpu/run.sh r06_y hot || exit $?
echo done
