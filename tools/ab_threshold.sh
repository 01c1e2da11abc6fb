# Exact-replay threshold sweep on the C3 bench (step time, bit-exact share, max rank error)
export TMPDIR=/tmp; mkdir -p gpurun_out
for t in ${TS:-32768 24576 16384}; do
  timeout -k 10 400 python -u bench.py --steps 10 --exact-threshold $t > gpurun_out/thr_$t.json 2>gpurun_out/thr_$t.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/thr_$t.json')); p=d['parity']; print('thr=$t', round(d['value']/1e9,3), round(d['ms_per_step'],3), p['quantiles_bit_exact_frac'], p['rank_error_max'])"
done
