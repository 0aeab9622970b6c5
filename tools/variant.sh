#!/bin/bash
# Build an experiment variant of libshirley_rt.so into exp/<name>/ (for tools/gpu.sh ab steps).
# Usage: tools/variant.sh <name> [extra hipcc flags...]   e.g. tools/variant.sh phase -DRT_PHASE_TIMING
# The tree is copied, so a variant can also be made from edited sources: set SRC=<dir> (default: the
# in-tree package).  LICM_FLAG= (empty) builds without -disable-machine-licm; TRK_FLAG=<flags> adds scheduler flags.
set -e
cd "$(dirname "$0")/.."
name=$1; shift
src=${SRC:-shirley-raytracing-rs_amd}
tmp=/tmp/variant_$name
rm -rf "$tmp" && mkdir -p "$tmp"
cp -r "$src"/csrc "$src"/Makefile "$tmp"/
mkdir -p "$tmp/../include" 2>/dev/null || true
cp -r include "$tmp/../" 2>/dev/null || true
make -C "$tmp" -j8 lib/libshirley_rt.so ARCH="${ARCH:-gfx950}" \
  HIPFLAGS="--offload-arch=${ARCH:-gfx950} -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wall -Wno-unused-function ${LICM_FLAG--mllvm -disable-machine-licm} ${TRK_FLAG-} $*" >/dev/null
mkdir -p exp/$name
cp "$tmp/lib/libshirley_rt.so" exp/$name/
cp shirley-raytracing-rs_amd/lib/libshirley_host.so exp/$name/
echo "exp/$name/libshirley_rt.so"
