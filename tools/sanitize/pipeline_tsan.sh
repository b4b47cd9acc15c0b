#!/bin/bash
# ThreadSanitizer build + run of the host frame pipeline (csrc/host/pipeline.cpp).
#   bash tools/sanitize/pipeline_tsan.sh [out_dir] [rounds]
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${1:-$ROOT/build/sanitize}"
mkdir -p "$OUT"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread -I"$ROOT/csrc/include" \
  "$ROOT/csrc/host/pipeline.cpp" "$ROOT/tools/sanitize/pipeline_stress.cpp" -pthread -o "$OUT/pipeline_stress"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/pipeline_stress" "${2:-300}"
