#!/bin/bash
# Build an experiment variant of libavse_hip.so into expso/<name>.so from a PATCHED COPY of the kernel sources:
# the product sources carry no experiment switches.  PATCH is a unified diff (git diff format, paths relative to the
# repo root) applied to the copy, e.g. one that compiles out the scan backward's dB/dC reduction for an A/B timing.
# usage: tools/build_exp.sh NAME [PATCH] ["-DFLAG ..."]
set -e
name=$1; patch=${2:-}; flags=${3:-}
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/build/exp/$name/src
out=$root/build/exp/$name
rm -rf "$src"; mkdir -p "$src/avse_challenge_amd" "$root/expso"
cp -r "$root/avse_challenge_amd/csrc" "$src/avse_challenge_amd/"      # same relative layout: common.h includes
cp -r "$root/include" "$src/"                                        # ../../include/avse_hip.h
if [ -n "$patch" ]; then
    (cd "$src" && patch -p1 < "$root/$patch")
fi
status=0
for f in "$src"/avse_challenge_amd/csrc/*.hip; do
    extra=""; [ "$(basename "$f")" = scan.hip ] && extra="-fno-slp-vectorize"    # as the Makefile builds it
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I"$src/include" $extra $flags -c "$f" \
        -o "$out/$(basename "$f" .hip).o" &
done
for j in $(jobs -p); do wait "$j" || status=1; done
[ $status -eq 0 ] || { echo "compile failed"; exit 1; }
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/expso/$name.so" "$out"/*.o
echo "built expso/$name.so"
