#!/bin/bash
# Build libapn_hip.so from a source directory (e.g. an older revision's csrc copied out of git)
# into ab/<name>/libapn_hip.so. Usage: tools/ab_build_src.sh <name> <csrc dir> ["<extra hipcc flags>"]
set -e
name=$1; src=$2; flags=$3
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/ab/$name; mkdir -p $out/build
objs=""
for f in $src/*.hip $src/apn_version.cpp; do
  b=$(basename $f); o=$out/build/${b%.*}.o
  extra="-fno-slp-vectorize -Xclang -target-feature -Xclang -packed-fp32-ops"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off $extra $flags -c $f -o $o &
  objs="$objs $o"
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $objs -o $out/libapn_hip.so
rm -rf $out/build
echo "built $out/libapn_hip.so from $src ($flags)"
