# C2 groups interleaved per queue entry (VN_C2_GROUPS 3, 4 against 2): batched-replay tests, 17M key
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-c2g}
for v in _g3 _g4 ""; do
  VN_LIB=libveneur_amd$v.so timeout -k 10 300 python -u -m pytest tests/test_batch_replay_gpu.py -x -q --timeout 150 --timeout-method thread > gpurun_out/${T}${v}_tests.log 2>&1 || exit 1
  VN_LIB=libveneur_amd$v.so timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}${v}_hot.log 2>&1 || exit 1
  echo "$v $(tail -n 1 gpurun_out/${T}${v}_hot.log)"
done
echo "rc=0"
