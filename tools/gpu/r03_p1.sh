set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VN_LIB=libveneur_amd_prof.so timeout -k 10 300 python -u tools/exact_profile.py 1000000 4000000 > gpurun_out/r03_p1.log 2>&1
echo "rc=$?"
