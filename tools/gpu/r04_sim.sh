# per-rank window time of an N-GPU split, one rank at a time on this GPU (bench.py --sim-world);
# usage: r04_sim.sh TAG N "ranks" [bench args...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=${HWQ:-16}
T=$1; N=$2; R=$3; shift 3
for r in $R; do
  timeout -k 10 200 python -u bench.py --sim-world $N --sim-rank $r --steps 8 --warmup 1 --c5-hosts 0 \
    --text-lines 0 --timing-steps 0 --pcie-steps 0 "$@" > gpurun_out/${T}_${N}_${r}.json 2> gpurun_out/${T}_${N}_${r}.log || exit 1
  echo "N=$N r=$r done"
done
echo "rc=0"
