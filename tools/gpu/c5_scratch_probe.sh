set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r05_c5x
A="--c5-only --c5-parity-keys 16"
timeout -k 10 200 python -u bench.py $A > ${O}_plain.json 2> ${O}_plain.log &&
HSA_SCRATCH_SINGLE_LIMIT=1048576 timeout -k 10 300 python -u bench.py $A > ${O}_smallscratch.json 2> ${O}_smallscratch.log &&
(cd /tmp && HSA_SCRATCH_SINGLE_LIMIT=8589934592 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/${O}_prof_bigscratch -o run -- python3 $GRAFT_REPO_ROOT/bench.py $A > $GRAFT_REPO_ROOT/${O}_prof_bigscratch.log 2>&1)
echo rc=$?
