set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
( for i in $(seq 1 60); do date +%s.%N; rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|fclk|mclk" ; sleep 0.5; done ) > gpurun_out/r04_g7_smi.log 2>&1 &
SMI=$!
timeout -k 10 300 python -u bench.py --c5-hosts 0 --text-lines 0 --no-cpu-baseline --steps 30 --timing-steps 0 --pcie-steps 0 --pipeline 2 > gpurun_out/r04_g7.json 2> gpurun_out/r04_g7.log
rc=$?
kill $SMI 2>/dev/null
echo "rc=$rc"
