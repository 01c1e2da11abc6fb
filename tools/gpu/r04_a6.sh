set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for lib in libveneur_amd.so libveneur_amd_variant.so libveneur_amd_dbg.so; do
VN_LIB=$lib timeout -k 10 120 python -u tools/debug_repeat.py debug/debug_rising.npz 25362 4 2>&1 | grep -v amdgpu.ids | cut -c1-600 || exit 1
done > gpurun_out/r04_a6.log 2>&1
echo "rc=$?"
