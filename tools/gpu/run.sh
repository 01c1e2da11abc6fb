#!/bin/bash
# The one GPU-box script: every gpurun call of the build runs one or more of its steps.
#   gpurun -- bash tools/gpu/run.sh TAG STEP [STEP ...]
# Steps (outputs under gpurun_out/TAG_*):
#   tests    every -m gpu test (stops the call at the first failure)
#   smoke    __graft_entry__.smoke()
#   bench    the default bench line (python bench.py)
#   bench1   the bench with one engine (--pipeline 1), windows back to back
#   benchq   the default bench line without the CPU baseline / parity / C5 / text legs (timing only)
#   benchq4  benchq with four engines
#   benchqvar  the same with the A/B variant library (VN_LIB=libveneur_amd_variant.so)
#   prof     rocprofv3 --kernel-trace --stats of a short bench with ONE engine, so every kernel's
#            duration is its own (no other window's kernels beside it); roofline_check over it
#   c5       the C5 leg alone (bench.py --c5-only)
#   c5prof   rocprofv3 --kernel-trace --stats of the C5 leg alone (16 hardware queues, as bench.py sets)
#   c5prof4  the same with HIP's default 4 hardware queues
#   c5profvar / c5var  the C5 leg with the A/B variant library, under the profiler / alone
#   pmc      FETCH_SIZE and WRITE_SIZE passes (separate runs) for the replay's HBM traffic
#   pmcvar   the same with the A/B variant library
#   c5setprof  k_set_merge cycles per payload kind over the C5 leg (variant built with -DVN_SET_PROF)
#   setprof  k_set_segments phase cycles (variant library built with -DVN_SET_PROF)
#   sim-N-R-D  rank R of an N-GPU C4 window alone, D engines in turn (bench.py --sim-world N --sim-rank R)
#   hot      batched-replay parity tests, phase cycles (profiling build) and the 17M-sample key
#   short    the one-wave replay's throughput (20k keys of 6000 samples, C5's per-drain size)
#            with this build and with the A/B variant library; then 64 such keys checked
# Each step runs under its own time limit; the first failure, fault, abort or timeout ends
# the call (no retries).
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=$1
shift
O=gpurun_out/$TAG
SHORT="--steps 2 --warmup 1 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --parity-keys 64"
for step in "$@"; do
  echo "[run.sh] $TAG: $step ($(date +%T))"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > ${O}_tests.log 2>&1 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > ${O}_smoke.txt 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py > ${O}_bench.json 2> ${O}_bench.log ;;
    bench1)
      timeout -k 10 600 python -u bench.py --pipeline 1 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 \
        --text-lines 0 > ${O}_bench1.json 2> ${O}_bench1.log ;;
    benchq)
      timeout -k 10 400 python -u bench.py --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 \
        > ${O}_benchq.json 2> ${O}_benchq.log ;;
    benchq4)
      timeout -k 10 400 python -u bench.py --pipeline 4 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 \
        > ${O}_benchq4.json 2> ${O}_benchq4.log ;;
    benchqvar)
      VN_LIB=libveneur_amd_variant.so timeout -k 10 400 python -u bench.py --no-cpu-baseline --pcie-steps 0 \
        --c5-hosts 0 --text-lines 0 > ${O}_benchqvar.json 2> ${O}_benchqvar.log ;;
    prof)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/${O}_prof" \
        -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --pipeline 1 $SHORT > "$GRAFT_REPO_ROOT/${O}_prof.log" 2>&1) &&
      python3 tools/roofline_check.py ${O}_prof ${O}_prof.log 1 ${O}_timing_step_kernel_stats.csv \
        > ${O}_roofline_check.txt 2>&1 ;;
    c5prof4)
      (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/${O}_c5prof4" \
        -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --c5-only > "$GRAFT_REPO_ROOT/${O}_c5prof4.log" 2>&1) ;;
    c5profvar)
      (cd /tmp && VN_LIB=libveneur_amd_variant.so timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$GRAFT_REPO_ROOT/${O}_c5profvar" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --c5-only \
        > "$GRAFT_REPO_ROOT/${O}_c5profvar.log" 2>&1) ;;
    c5var)
      VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u bench.py --c5-only > ${O}_c5var.json 2> ${O}_c5var.log ;;
    c5)
      timeout -k 10 300 python -u bench.py --c5-only > ${O}_c5.json 2> ${O}_c5.log ;;
    c5prof)
      # (bench.py sets GPU_MAX_HW_QUEUES=16 before HIP starts, but under the profiler HIP is up before
      # bench.py runs: with the default 4 queues the engine's streams share hardware queues, and a
      # CU-masked stream's mask then holds the replays sharing its queue)
      (cd /tmp && GPU_MAX_HW_QUEUES=16 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/${O}_c5prof" \
        -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --c5-only > "$GRAFT_REPO_ROOT/${O}_c5prof.log" 2>&1) ;;
    pmc)
      A="--steps 1 --warmup 0 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --parity-keys 64"
      timeout -k 10 300 python bench.py $A > ${O}_pmcbench.json 2> ${O}_pmcbench.log &&
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/${O}_fetch" -o run \
        -- python3 "$GRAFT_REPO_ROOT/bench.py" $A > "$GRAFT_REPO_ROOT/${O}_fetch.log" 2>&1) &&
      (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$GRAFT_REPO_ROOT/${O}_write" -o run \
        -- python3 "$GRAFT_REPO_ROOT/bench.py" $A > "$GRAFT_REPO_ROOT/${O}_write.log" 2>&1) ;;
    pmcvar)
      # the pmc passes with the A/B variant library
      A="--steps 1 --warmup 0 --timing-steps 1 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --parity-keys 64"
      VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python bench.py $A > ${O}_pmcvarbench.json 2> ${O}_pmcvarbench.log &&
      (cd /tmp && VN_LIB=libveneur_amd_variant.so timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d "$GRAFT_REPO_ROOT/${O}_varfetch" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $A > "$GRAFT_REPO_ROOT/${O}_varfetch.log" 2>&1) &&
      (cd /tmp && VN_LIB=libveneur_amd_variant.so timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv \
        -d "$GRAFT_REPO_ROOT/${O}_varwrite" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" $A > "$GRAFT_REPO_ROOT/${O}_varwrite.log" 2>&1) ;;
    hot)
      timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py -x -q --timeout 150 --timeout-method thread \
        > ${O}_hot_tests.log 2>&1 &&
      VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 > ${O}_hot_prof.log 2>&1 &&
      timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > ${O}_hot_17M.log 2>&1 ;;
    short)
      H="tools/hot_replay_bench.py --n 6000 --keys 1 --cold-keys 20000 --cold-n 6000 --no-check --reps 3"
      timeout -k 10 200 python -u $H > ${O}_short.log 2>&1 &&
      VN_LIB=libveneur_amd_variant.so timeout -k 10 200 python -u $H > ${O}_short_var.log 2>&1 &&
      timeout -k 10 200 python -u tools/hot_replay_bench.py --n 6000 --keys 64 --reps 1 > ${O}_short_check.log 2>&1 ;;
    setprof)
      # (needs the variant library built with VARIANT_FLAGS=-DVN_SET_PROF)
      VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u tools/set_profile.py > ${O}_setprof.log 2>&1 ;;
    c5setprof)
      # (needs the variant library built with VARIANT_FLAGS=-DVN_SET_PROF)
      VN_LIB=libveneur_amd_variant.so timeout -k 10 300 python -u tools/c5_set_profile.py > ${O}_c5setprof.log 2>&1 ;;
    shortprof)
      # the one-wave replay's phase split (profiling build): 6000-sample keys, alone and with 20k beside
      VN_LIB=libveneur_amd_prof.so timeout -k 10 200 python -u tools/exact_profile.py short:6000:0 short:6000:20000 \
        > ${O}_shortprof.log 2>&1 ;;
    simlib:*)
      # simlib:LIB:N:R:D -- the per-rank C4 sim with libveneur_amd_LIB.so (LIB "main": the product)
      IFS=: read -r _ SL SN SR SD <<< "$step"
      LIBV=libveneur_amd_$SL.so; [ "$SL" = main ] && LIBV=libveneur_amd.so
      VN_LIB=$LIBV timeout -k 10 400 python -u bench.py --sim-world $SN --sim-rank $SR --pipeline $SD \
        --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 \
        > ${O}_simlib_${SL}_${SN}_${SR}_${SD}.json 2> ${O}_simlib_${SL}_${SN}_${SR}_${SD}.log ;;
    batchlib:*)
      # batchlib:LIB -- the batched replay's first whole-digest test with that library; an assertion
      # failure is reported and the call goes on, a GPU fault ends it
      IFS=: read -r _ SL <<< "$step"
      VN_LIB=libveneur_amd_$SL.so timeout -k 10 200 python -u -m pytest \
        "tests/test_batch_replay_gpu.py::test_batched_replay_whole_digest_bit_exact[1]" -x -q --timeout 150 \
        --timeout-method thread > ${O}_batchlib_$SL.log 2>&1
      echo "[run.sh] batchlib $SL pytest rc=$?"
      if grep -q "illegal memory access\|Memory access fault\|Aborted" ${O}_batchlib_$SL.log; then (exit 3); else (exit 0); fi ;;
    testlib:*)
      # testlib:LIB:TESTID -- one test with libveneur_amd_LIB.so ("main": the product); an assertion
      # failure is reported and the call goes on, a GPU fault ends it
      IFS=: read -r _ SL ST <<< "$step"
      LIBV=libveneur_amd_$SL.so; [ "$SL" = main ] && LIBV=libveneur_amd.so
      VN_LIB=$LIBV timeout -k 10 300 python -u -m pytest "$ST" -x -q --timeout 250 --timeout-method thread \
        > ${O}_testlib_${SL}.log 2>&1
      echo "[run.sh] testlib $SL pytest rc=$?"
      if grep -q "illegal memory access\|Memory access fault\|Aborted" ${O}_testlib_${SL}.log; then (exit 3); else (exit 0); fi ;;
    sim-*|simvar-*)
      # sim-N-R-D: rank R of an N-GPU C4 run alone on this GPU, D engines in turn (bench.py --sim-world)
      # sim-N-R-D-C-Q: C CUs reserved for the longest replays, Q hardware queues (defaults 0, 16);
      # simvar-...: the same with the A/B variant library
      IFS=- read -r SK SN SR SD SC SQ <<< "$step"
      SC=${SC:-0}; SQ=${SQ:-16}
      LIBV=libveneur_amd.so; [ "$SK" = simvar ] && LIBV=libveneur_amd_variant.so
      VN_LIB=$LIBV GPU_MAX_HW_QUEUES=$SQ timeout -k 10 400 python -u bench.py --sim-world $SN --sim-rank $SR \
        --pipeline $SD --reserved-cus $SC --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 \
        > ${O}_${SK}_${SN}_${SR}_${SD}_${SC}_${SQ}.json 2> ${O}_${SK}_${SN}_${SR}_${SD}_${SC}_${SQ}.log ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
  rc=$?
  echo "[run.sh] $TAG: $step rc=$rc ($(date +%T))"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
exit 0
