set -o pipefail
cd $GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_LDS -d gpurun_out/r03_pmc_lds -o pmc -- python3 tools/hot_replay_bench.py --n 1000000 --keys 1 --reps 1 --no-check > gpurun_out/r03_pmc_lds.log 2>&1
echo done
