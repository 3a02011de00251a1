#!/bin/bash
# Build the working tree's HIP shim with one source edit applied to a copy, into
# uigc-akka_amd/lib/ab/<name>.so (experiments for tools/gpu_ab2.sh; the tree
# itself is not touched).  Runs here, on the CPU.
# usage: bash tools/build_variant.sh <name> <file.hip> <python-replace-script | ->
#   the script reads the source from stdin and writes the edited one to stdout
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1
FILE=$2
EDIT=$3
T=$(mktemp -d)
mkdir -p "$T/a"
cp -r "$ROOT/uigc-akka_amd/csrc" "$T/a/csrc"  # csrc/../../include is $T/include
mkdir -p "$T/include" "$T/obj" "$ROOT/uigc-akka_amd/lib/ab"
cp "$ROOT/include/crgc.h" "$T/include/"
# EDIT "-": the working tree as it is
[ "$EDIT" != "-" ] && python3 -c "$EDIT" < "$ROOT/uigc-akka_amd/csrc/$FILE" > "$T/a/csrc/$FILE"
if [ "$EDIT" != "-" ] && cmp -s "$ROOT/uigc-akka_amd/csrc/$FILE" "$T/a/csrc/$FILE"; then
  echo "edit changed nothing" >&2
  exit 1
fi
FLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -w -munsafe-fp-atomics"
pids=()
for s in "$T"/a/csrc/*.hip; do
  /opt/rocm/bin/hipcc $FLAGS -c "$s" -o "$T/obj/$(basename "$s" .hip).o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/uigc-akka_amd/lib/ab/$NAME.so" "$T"/obj/*.o \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
rm -rf "$T"
echo "$ROOT/uigc-akka_amd/lib/ab/$NAME.so"
