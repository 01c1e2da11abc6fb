set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
(echo "== fast-merge-off variant"; VN_LIB=libveneur_amd_variant.so timeout -k 10 120 python -u tools/debug_rising.py --kind rising --n 300000 --seed 1;
 echo "== default"; timeout -k 10 200 python -u tools/debug_rising.py --kind rising --n 300000 --seed 1) > gpurun_out/r04_a3.log 2>&1
echo "rc=$?"
