#!/bin/bash
# Build an experiment variant of the engine for timing (tools/iterbench.py):
#   bash tools/build_variant.sh <name> <engine source> [extra hipcc flags]
# -> mpc-tsid_amd/csrc/build/variants/libmpcq_<name>.so (loaded with
#    MPCQ_LIB_VARIANT=exp:<name>); only the horizons $VARIANT_HORIZONS (default 16 32),
#    from the variant source, the rest of the library from the current objects (run
#    make first).
#   bash tools/build_variant.sh --stamp-only <name> <engine source> [flags]: print the stamp
# The library reports its own build stamp (mpcq_build_info): the production stamp, then
# "+exp:<name>:<12 hex of sha256 over the variant source, its flags and horizons>", so
# bench.py never quotes production PMC figures (profiles/pmc_traffic.json) for a variant.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/mpc-tsid_amd/csrc
STAMP_ONLY=0
if [ "$1" = "--stamp-only" ]; then STAMP_ONLY=1; shift; fi
NAME=$1; SRC=$(realpath "$2"); shift 2
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -I$C"
HS=${VARIANT_HORIZONS:-16 32}  # the horizons compiled from the variant source
VH=$( (cat "$SRC"; printf '%s|' "$F" "$*" "$HS" "${NOELIDE:-}") | sha256sum | cut -c1-12)
VSHA="$(python3 $C/stamp.py)+exp:$NAME:$VH"
if [ $STAMP_ONLY = 1 ]; then echo "$VSHA"; exit 0; fi
OUT=$C/build/variants; mkdir -p $OUT/$NAME
J=0
CC=/opt/rocm/bin/hipcc
# through the production build's nop-elision pass (csrc/asmpass) unless NOELIDE=1
if [ -z "$NOELIDE" ]; then CC="python3 $C/asmpass/hipcc_elide.py"; fi
for n in $HS; do
  $CC $F "$@" -DMPCQ_ENGINE_N=$n -c -o $OUT/$NAME/e$n.o -x hip $SRC &
  J=$((J + 1)); if [ $((J % 8)) -eq 0 ]; then wait; fi
done
wait
# only the variant's horizons (a dispatch unit restricted to them: the library stays
# small, every gpurun call ships it)
OBJS=""
HX=""
for n in $HS; do OBJS="$OBJS $OUT/$NAME/e$n.o"; HX="$HX X($n)"; done
printf '#include "mpcq_internal.h"\n#undef MPCQ_HORIZONS\n#define MPCQ_HORIZONS(X) %s\n#include "mpcq_dispatch.cpp"\n' "$HX" > $OUT/$NAME/dispatch.cpp
/opt/rocm/bin/hipcc $F "$@" -I$R/include -c -o $OUT/$NAME/dispatch.o $OUT/$NAME/dispatch.cpp
# the C ABI with the variant's flags too (a layout switch changes work_doubles)
/opt/rocm/bin/hipcc $F "$@" -I$R/include -c -o $OUT/$NAME/api.o $C/mpcq_api.cpp
# the variant's own build stamp
/opt/rocm/bin/hipcc $F -DMPCQ_SRC_SHA="\"$VSHA\"" -DMPCQ_ARCH='"gfx950"' -c -o $OUT/$NAME/build.o $C/mpcq_build.cpp
/opt/rocm/bin/hipcc $F -shared -o $OUT/libmpcq_$NAME.so $OBJS $C/build/mpcq_planner.o $C/build/mpcq_session.o $C/build/mpcq_order.o \
  $OUT/$NAME/api.o $OUT/$NAME/build.o $OUT/$NAME/dispatch.o
echo "built $OUT/libmpcq_$NAME.so"
