set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in prof prof_nowelf prof_nofetch; do echo "== $v"; VN_LIB=libveneur_amd_$v.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 || exit 1; done > gpurun_out/r03_p2.log 2>&1
echo "rc=$?"
