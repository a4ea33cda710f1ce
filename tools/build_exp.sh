#!/bin/bash
# Build experiment variants of libavse_hip.so into build/exp/<name>.so with extra -D flags.
# usage: tools/build_exp.sh NAME "-DFLAG1 -DFLAG2"
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/build/exp/$name
mkdir -p "$out" "$root/expso"
for f in "$root"/avse_challenge_amd/csrc/*.hip; do
    extra=""; [ "$(basename "$f")" = scan.hip ] && extra="-fno-slp-vectorize"    # as the Makefile builds it
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -I"$root/include" $extra $flags -c "$f" -o "$out/$(basename "$f" .hip).o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/expso/$name.so" "$out"/*.o
echo "built expso/$name.so"
