#!/bin/bash
# Build a variant of libwcpt.so with extra compile flags, for A/B runs (tools/ab.py with WCPT_LIBRARY=...).
#   bash tools/ab_build.sh NAME "-DWCPT_MK_WAVES=5"   -> wc-path-tracer_amd/variants/NAME.so
set -e
cd "$(dirname "$0")/../wc-path-tracer_amd"
mkdir -p variants
make -j8 BUILD=build_$1 LIB=variants/$1.so EXTRA="$2" >/dev/null
echo "wc-path-tracer_amd/variants/$1.so"
