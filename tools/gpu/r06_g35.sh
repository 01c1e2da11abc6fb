set -o pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; mkdir -p gpurun_out
T=r06_tl
Q="--no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --steps 8 --warmup 2 --parity-keys 64"
(cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/${T}_trace" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $Q > "$GRAFT_REPO_ROOT/gpurun_out/${T}_trace.log" 2>&1) || exit 11
echo done
