set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/r04_e1_tests.log 2>&1 &&
timeout -k 10 300 python -u tools/hot_replay_bench.py --n 17000000 --keys 1 --rates --reps 2 > gpurun_out/r04_e1_hot.log 2>&1 &&
timeout -k 10 900 python -u bench.py --c5-hosts 0 --text-lines 0 > gpurun_out/r04_e1_bench.json 2> gpurun_out/r04_e1_bench.log
echo "rc=$?"
