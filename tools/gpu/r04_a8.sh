set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
VN_LIB=libveneur_amd_prof.so timeout -k 10 120 python -u tools/exact_profile.py 4000000 > gpurun_out/r04_a8_prof.log 2>&1
echo "rc=$?"
