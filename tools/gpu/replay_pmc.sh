# SQ counters of the batched replay of one 4M-sample key (one pass: 8 SQ counters): where the
# waves' cycles go (waiting at s_waitcnt / barriers, issue stalls, LDS bank conflicts)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05_pmc}
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_sq -o run -- python3 $GRAFT_REPO_ROOT/tools/hot_replay_bench.py --n 4000000 --keys 1 --reps 1 --no-check > $GRAFT_REPO_ROOT/gpurun_out/${T}_sq.log 2>&1) &&
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_UNALIGNED_STALL --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_sq2 -o run -- python3 $GRAFT_REPO_ROOT/tools/hot_replay_bench.py --n 4000000 --keys 1 --reps 1 --no-check > $GRAFT_REPO_ROOT/gpurun_out/${T}_sq2.log 2>&1)
