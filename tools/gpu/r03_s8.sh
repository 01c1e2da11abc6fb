set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u tools/c4_histo_replay.py > gpurun_out/r03_c4h.log 2>&1
echo done
