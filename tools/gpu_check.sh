#!/bin/bash
# GPU-box check: parity tests, bench, rocprof kernel stats.  Stops at the first step that
# fails, faults, aborts or times out.
#   tools/gpu_check.sh TAG [skip-tests|tests] [pmc]
export TMPDIR=/tmp
TAG=${1:-run}
mkdir -p gpurun_out
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc" >> gpurun_out/${TAG}_tests.log
  if [ $rc -ne 0 ]; then exit $rc; fi  # a failed test may be a device fault: stop here
fi
timeout -k 10 400 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.log || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- \
  python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python3 tools/roofline_check.py gpurun_out/${TAG}_prof gpurun_out/${TAG}_prof.log 1 gpurun_out/${TAG}_timing_step_kernel_stats.csv > gpurun_out/${TAG}_roofline_check.txt 2>&1
if [ "$3" = "pmc" ]; then
  # HBM traffic: FETCH_SIZE and WRITE_SIZE in separate passes (TCC slots), counters only
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_fetch -o run -- \
    python3 bench.py --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc_fetch.log 2>&1 || exit $?
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_pmc_write -o run -- \
    python3 bench.py --steps 1 --warmup 1 --timing-steps 1 --no-cpu-baseline > gpurun_out/${TAG}_pmc_write.log 2>&1 || exit $?
fi
exit 0
