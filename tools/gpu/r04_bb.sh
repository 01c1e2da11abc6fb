# batch size A/B on the 17M-sample key (bit-exactness checked by the tool)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-bb}
for v in "" _bb48 _bb40; do
  VN_LIB=libveneur_amd$v.so timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/${T}$v.log 2>&1 || exit 1
  tail -n 1 gpurun_out/${T}$v.log
done
echo "rc=0"
