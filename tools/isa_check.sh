#!/bin/bash
# Scan the gfx950 code objects of the built library's objects for scalar-cache writes
# (scalar stores / atomics / write-back / discard), which this project never emits.
set -e
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
bad=0
for o in "$(dirname "$0")"/../veneur_amd/build/*.o; do
  n=$(basename "$o" .o)
  "$B/llvm-objcopy" --dump-section .hip_fatbin="$T/$n.fatbin" "$o" 2>/dev/null || continue
  tgt=$("$B/clang-offload-bundler" --list --type=o --input="$T/$n.fatbin" | grep gfx950)
  "$B/clang-offload-bundler" --unbundle --type=o --input="$T/$n.fatbin" --targets="$tgt" --output="$T/$n.co"
  c=$("$B/llvm-objdump" -d "$T/$n.co" | grep -cE 's_store|s_atomic|s_dcache_wb|s_buffer_store|s_dcache_discard' || true)
  echo "$n: $c"
  [ "$c" = "0" ] || bad=1
done
rm -rf "$T"
exit $bad
