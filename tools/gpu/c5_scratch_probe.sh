# C5 under the profiler with 4 hardware queues (r05_c5y: a malformed-payload error there before
# vn_device_copy waited for its copy), then the same with bench's default of 16 queues
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_c5z
A="--c5-only --c5-parity-keys 16"
(cd /tmp && GPU_MAX_HW_QUEUES=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/${O}_prof_hwq4 -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/${O}_prof_hwq4.log 2>&1)
