#!/bin/bash
# ThreadSanitizer build + run of the timed-region copy pool (csrc/runtime/hostcopy.cpp) under back-to-back runs.
#   bash tools/sanitize/hostcopy_tsan.sh [out_dir] [iters]
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${1:-$ROOT/build/sanitize}"
mkdir -p "$OUT"
g++ -std=c++17 -O1 -g -fno-omit-frame-pointer -fsanitize=thread -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include \
  -I"$ROOT/csrc/include" "$ROOT/csrc/runtime/hostcopy.cpp" "$ROOT/csrc/runtime/log.cpp" \
  "$ROOT/tools/sanitize/hostcopy_stress.cpp" -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lrocprofiler-sdk-roctx -pthread \
  -o "$OUT/hostcopy_stress"
TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1 "$OUT/hostcopy_stress" "${2:-20000}" 3
