#!/bin/bash
# Build the HIP shim of a git revision into uigc-akka_amd/lib/ab/<name>.so (for
# CRGC_LIB_AB A/Bs against the in-tree build).  Runs here, on the CPU.
# usage: bash tools/build_ab.sh <rev> <name>
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
REV=$1
NAME=$2
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" uigc-akka_amd/csrc include | tar -x -C "$T"
mkdir -p "$ROOT/uigc-akka_amd/lib/ab" "$T/obj"
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -munsafe-fp-atomics"
pids=()
for s in "$T"/uigc-akka_amd/csrc/*.hip; do
  /opt/rocm/bin/hipcc $FLAGS -c "$s" -o "$T/obj/$(basename "$s" .hip).o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/uigc-akka_amd/lib/ab/$NAME.so" "$T"/obj/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "$ROOT/uigc-akka_amd/lib/ab/$NAME.so"
