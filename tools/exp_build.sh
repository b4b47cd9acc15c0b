#!/bin/bash
# Build an experimental variant of libstereo_amd.so with extra -D flags on the conv kernel (kernel A/B
# experiments; load it with SA_NATIVE_LIB=<path>).  Everything else links the normal objects.
#   bash tools/exp_build.sh <name> -DSA_EXP_FOO ...
set -eo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
name=$1; shift
out="$ROOT/stereoalgorithms_amd/lib/exp"
mkdir -p "$out" "$ROOT/build/exp"
obj="$ROOT/build/exp/conv2d_$name.o"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -std=c++17 -fPIC -I"$ROOT/csrc/include" -I"$ROOT/csrc/models" \
  -munsafe-fp-atomics "$@" -c "$ROOT/csrc/kernels/conv2d.hip" -o "$obj"
objs=$(ls "$ROOT"/build/obj/dev/*.o | grep -v "/conv2d.hip.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o "$out/libstereo_amd_$name.so" $objs "$obj" \
  -L"$ROOT/stereoalgorithms_amd/lib" -lstereo_host -Wl,-rpath,'$ORIGIN/..' -L/opt/rocm/lib -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib
echo "$out/libstereo_amd_$name.so"
