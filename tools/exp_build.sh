#!/bin/bash
# Build an experimental variant of libstereo_amd.so (kernel A/B experiments; load it with SA_NATIVE_LIB=<path>).
# One kernel source is recompiled -- with extra -D flags, or replaced by another file -- and everything else links
# the normal objects.
#   bash tools/exp_build.sh <name> [-DSA_EXP_FOO ...]                      (variant of conv2d.hip)
#   SRC=csrc/kernels/motion_enc.hip ALT=/tmp/old.hip bash tools/exp_build.sh <name>   (ALT compiled in SRC's place)
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; shift
SRC=${SRC:-csrc/kernels/conv2d.hip}
ALT=${ALT:-$ROOT/$SRC}
base=$(basename "$SRC")
out="$ROOT/stereoalgorithms_amd/lib/exp"
mkdir -p "$out" "$ROOT/build/exp"
obj="$ROOT/build/exp/${base%.hip}_$name.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -fPIC -I"$ROOT/csrc/include" -I"$ROOT/csrc/models" \
  -munsafe-fp-atomics "$@" -c "$ALT" -o "$obj"
objs=$(ls "$ROOT"/build/obj/dev/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libstereo_amd_$name.so" $objs "$obj" \
  -L"$ROOT/stereoalgorithms_amd/lib" -lstereo_host -Wl,-rpath,'$ORIGIN/..' -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$out/libstereo_amd_$name.so"
