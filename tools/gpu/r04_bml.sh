# batched-replay minimum key length A/B: C5 (one drain and 64Mi drains) and C4 (three engines)
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${1:-bml}
for v in bml16 bml8; do
  VN_LIB=libveneur_amd_$v.so timeout -k 10 400 python -u tools/c5_check.py 1000,10000,2000,67108864 1000,10000,2000,805306368 > gpurun_out/${T}_${v}_c5.log 2>&1 || exit 1
  VN_LIB=libveneur_amd_$v.so timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline --pcie-steps 0 --c5-hosts 0 --text-lines 0 --parity-keys 3000 > gpurun_out/${T}_${v}_c4.json 2> gpurun_out/${T}_${v}_c4.log || exit 1
done
echo "rc=0"
