#!/bin/bash
# Build tuning variants of the scan kernels in parallel (the sequential
# `make variants` takes ~2.5 min per variant):
#   tools/build_variants.sh 'name=-DKNOB=1 -DOTHER=2' 'name2=...' ...
# Writes distributed-grep_amd/variants/libdgrep_<name>.so (run with
# DGREP_LIB=...; tools/variant_bench.sh). The other objects come from the
# normal build, which must be current (make -C distributed-grep_amd).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/distributed-grep_amd
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function"
mkdir -p "$P/variants" "$P/build"
make -s -C "$P" >/dev/null
pids=()
for spec in "$@"; do
  name=${spec%%=*}
  defs=${spec#*=}
  (
    # the runtime builds the LDS images, so it takes the same knobs
    # the scan kernels' build parts in parallel (see scan_dfa.hip), then the runtime
    # PARTS (default all): the scan build parts this variant recompiles; the
    # others are linked from the normal build
    pp=()
    for k in 0 1 2 3 4; do
      if [[ " ${PARTS:-0 1 2 3 4} " == *" $k "* ]]; then
        $HIPCC $FLAGS $defs -DDGREP_SCAN_PART=$k -c "$P/csrc/kernels/scan_dfa.hip" -o "$P/build/scan_dfa_${name}_p$k.o" 2> "$P/build/variant_${name}_p$k.log" &
        pp+=($!)
      else
        cp "$P/build/scan_dfa_p$k.o" "$P/build/scan_dfa_${name}_p$k.o"
      fi
    done
    $HIPCC $FLAGS $defs -c "$P/csrc/runtime/dgrep_runtime.hip" -o "$P/build/dgrep_runtime_$name.o" 2> "$P/build/variant_$name.log"
    for q in "${pp[@]}"; do wait "$q"; done
    ls "$P"/build/scan_dfa_${name}_p{0,1,2,3,4}.o > /dev/null &&
      mkdir -p "$P/build/stamp_$name" &&
      sed "s|#define DGREP_BUILD_FLAGS \".*\"|#define DGREP_BUILD_FLAGS \"$defs\"|" "$P/build/build_stamp.h" > "$P/build/stamp_$name/build_stamp.h" &&
      g++ -O2 -std=c++17 -fPIC -I"$P/build/stamp_$name" -c "$P/csrc/runtime/build_info.cpp" -o "$P/build/build_info_$name.o" &&
      $HIPCC -shared -fPIC --offload-arch=gfx950 -o "$P/variants/libdgrep_$name.so" \
        "$P"/build/go_parser.o "$P"/build/dfa_builder.o "$P"/build/compile_api.o "$P"/build/scan_dfa_${name}_p{0,1,2,3,4}.o \
        "$P"/build/encode.o "$P"/build/reduce.o "$P/build/dgrep_runtime_$name.o" "$P"/build/exchange.o "$P/build/build_info_$name.o" \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib &&
      echo "built $name ($defs)"
  ) &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
exit $rc
