#!/bin/bash
# Build a variant of libcess_bls.so with extra -D flags, reusing the main
# build's objects for every translation unit except the ones listed.
# Usage: [MAKEVARS="FINAL_SCHED=max-ilp"] tools/build_variant.sh NAME "EXTRA FLAGS" k_final [k_pairing ...]
# Output: cess_amd/lib_variants/NAME/libcess_bls.so (select with CESS_BLS_LIB)
set -e
name=$1; extra=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
obj=$root/cess_amd/build_variants/$name
rm -rf "$obj"; mkdir -p "$obj"
cp -p "$root"/cess_amd/build/*.o "$obj"/
for k in "$@"; do rm -f "$obj/$k.o"; done
make -C "$root/cess_amd/csrc" -j8 OBJ="$obj" OUT="$root/cess_amd/lib_variants/$name" EXTRA="$extra" $MAKEVARS >/dev/null
ls -la "$root/cess_amd/lib_variants/$name/libcess_bls.so"
