#!/bin/bash
# Build the CPU-only host library sources with AddressSanitizer + UndefinedBehaviorSanitizer and run the
# host harness on the test fixtures (host code only: GPU sanitizers are not available on this pool).
#   bash tools/sanitize/run.sh [out_dir]
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${1:-$ROOT/build/sanitize}"
mkdir -p "$OUT"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined \
  -I"$ROOT/csrc/include" -I"$ROOT/csrc/abi" "$ROOT"/csrc/host/*.cpp "$ROOT/tools/sanitize/host_check.cpp" \
  -lz -o "$OUT/host_check"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 \
  "$OUT/host_check" "$ROOT/tests/fixtures" "$OUT"
