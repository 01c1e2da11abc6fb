# A/B of an engine environment switch on the C3 bench: tools/ab_env.sh VAR "v1 v2 ..." [parity]
# (with "parity" the CPU baseline runs too, and the full-scale parity summary is printed)
export TMPDIR=/tmp; mkdir -p gpurun_out
extra="--no-cpu-baseline"
[ "$3" = "parity" ] && extra=""
for v in $2; do
  env $1=$v timeout -k 10 400 python -u bench.py $extra --steps 10 > gpurun_out/ab_$1_$v.json 2>gpurun_out/ab_$1_$v.log || exit $?
  python -c "import json; d=json.load(open('gpurun_out/ab_$1_$v.json')); p=d.get('parity') or {}; print('$1=$v', round(d['value']/1e9,3), round(d['ms_per_step'],3), round(d['roofline']['achieved']), round(d['roofline']['frac'],3), p.get('quantiles_bit_exact_frac'), p.get('rank_error_max'))"
done
