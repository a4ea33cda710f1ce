#!/bin/bash
# Scan-only experiment builds: scan.hip with extra -D flags, linked with the in-tree objects of the other
# kernels (build/csrc/*.o from `make`).  usage: tools/build_scan_exp.sh NAME "-DFLAG ..."  -> expso/NAME.so
set -e
name=$1; flags=$2
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/build/exp/$name" "$root/expso"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -fno-slp-vectorize -I"$root/include" $flags \
    -c "$root/avse_challenge_amd/csrc/scan.hip" -o "$root/build/exp/$name/scan.o"
objs=$(ls "$root"/build/csrc/*.o | grep -v '/scan.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$root/expso/$name.so" $objs "$root/build/exp/$name/scan.o"
echo "built expso/$name.so"
