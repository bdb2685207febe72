#!/bin/bash
# Build a tuning variant of the library next to the product one:
#   tools/build_variant.sh NAME "-DPYAS_WAVES=8 ..."
# -> pyactivestorage_amd/lib/variants/libpyas_NAME.so (select with PYAS_LIB=...)
set -e
root=$(cd "$(dirname "$0")/.." && pwd)
make -C "$root/pyactivestorage_amd/csrc" -j"${MAX_JOBS:-8}" OBJDIR="$root/build/v_$1" \
    OUTDIR="$root/pyactivestorage_amd/lib/variants" LIBNAME="libpyas_$1.so" EXTRA="$2"
