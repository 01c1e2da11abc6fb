# which part of the profiling build changes the batched replay's decisions: 4M-sample key, bit-exactness and time
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-pd}
for v in "" _pA _pB _prof; do
  VN_LIB=libveneur_amd$v.so timeout -k 10 200 python -u tools/hot_replay_bench.py --n 4000000 --keys 1 --rates --reps 1 > gpurun_out/${T}$v.log 2>&1 || exit 1
  echo "$v $(tail -n 1 gpurun_out/${T}$v.log)"
done
echo "rc=0"
