# SQ counters of the exact replays (one pass of 8 SQ counters each): the batched replay of one
# 4M-sample key, and the one-wave replay of 100k short keys (300 samples each)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r05_pmc}
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_short -o run -- python3 $GRAFT_REPO_ROOT/tools/hot_replay_bench.py --n 300 --keys 1 --cold-keys 100000 --cold-n 300 --reps 1 --no-check > $GRAFT_REPO_ROOT/gpurun_out/${T}_short.log 2>&1) &&
(cd /tmp && timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${T}_short2 -o run -- python3 $GRAFT_REPO_ROOT/tools/hot_replay_bench.py --n 300 --keys 1 --cold-keys 100000 --cold-n 300 --reps 1 --no-check > $GRAFT_REPO_ROOT/gpurun_out/${T}_short2.log 2>&1)
