#!/bin/bash
# A/B of the product library against libveneur_amd_variant.so (make -C veneur_amd variant
# VARIANT_FLAGS=...): alternating C4 bench runs without the CPU legs; prints ms per window.
#   tools/ab_variant.sh TAG [rounds]
TAG=${1:-ab}; R=${2:-2}
mkdir -p gpurun_out
for i in $(seq 1 $R); do
  for v in base variant; do
    if [ $v = base ]; then lib=libveneur_amd.so; else lib=libveneur_amd_variant.so; fi
    VN_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --c5-hosts 0 --text-lines 0 \
      > gpurun_out/${TAG}_${v}_$i.json 2> gpurun_out/${TAG}_${v}_$i.log || exit $?
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'])" \
      gpurun_out/${TAG}_${v}_$i.json $v
  done
done
