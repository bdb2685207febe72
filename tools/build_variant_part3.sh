#!/bin/bash
# Like build_variant.sh, but reuses the product objects and rebuilds only the
# part-3 instantiations (the in-kernel fold launchers) with the variant flags:
#   tools/build_variant_part3.sh NAME "-DPYAS_LEAN_DEPTH=3 ..."
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$root/build/v_$1"
cp -p "$root"/build/pyas/*.o "$root/build/v_$1/"
rm -f "$root"/build/v_$1/inst_*_3.o
make -C "$root/pyactivestorage_amd/csrc" -j"${MAX_JOBS:-8}" OBJDIR="$root/build/v_$1" \
    OUTDIR="$root/pyactivestorage_amd/lib/variants" LIBNAME="libpyas_$1.so" EXTRA="$2"
