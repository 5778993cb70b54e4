#!/bin/bash
# Build the scan kernels + runtime of an older commit as a variant library
# (same box A/B against the working tree):
#   tools/build_commit_variant.sh <name> <commit> [extra -D flags]
# Writes distributed-grep_amd/variants/libdgrep_<name>.so; the compiler,
# encoder and reducer objects come from the current build.
set -euo pipefail
NAME=$1; COMMIT=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/distributed-grep_amd
W=$(mktemp -d /tmp/dgrep_wt.XXXX)
git -C "$R" worktree add -q --detach "$W" "$COMMIT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*"
mkdir -p "$P/variants"
make -s -C "$P" >/dev/null
$HIPCC $FLAGS -c "$W/distributed-grep_amd/csrc/kernels/scan_dfa.hip" -o "$P/build/scan_dfa_c_$NAME.o" 2> "$P/build/variant_$NAME.log" &
$HIPCC $FLAGS -c "$W/distributed-grep_amd/csrc/runtime/dgrep_runtime.hip" -o "$P/build/dgrep_runtime_c_$NAME.o" 2>> "$P/build/variant_$NAME.log" &
wait %1 && wait %2
$HIPCC -shared -fPIC --offload-arch=gfx950 -o "$P/variants/libdgrep_$NAME.so" "$P"/build/go_parser.o "$P"/build/dfa_builder.o \
  "$P"/build/compile_api.o "$P/build/scan_dfa_c_$NAME.o" "$P"/build/encode.o "$P"/build/reduce.o "$P/build/dgrep_runtime_c_$NAME.o" \
  "$P"/build/exchange.o "$P"/build/build_info.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
git -C "$R" worktree remove --force "$W"
echo "built $NAME from $COMMIT"
