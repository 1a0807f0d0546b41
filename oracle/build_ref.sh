#!/bin/bash
# Builds oracle/_ref/libsp_ref.so: the reference's own render path compiled from the sources
# under /root/reference (never copied), plus oracle/ref_harness.cpp (scene assembly + main.cpp's
# per-pixel loop).  TEST INFRASTRUCTURE ONLY; outputs go to oracle/_ref/ (git-ignored, travels
# to the GPU box with the snapshot).
#
# Flags: the reference's CMakeLists.txt builds with -std=gnu++20 -mfma -mavx2 and CMake's empty
# build type (no -O, hence no FP contraction).  -O2 -ffp-contract=off gives the same IEEE
# arithmetic.  The reference relies on transitively included standard headers that g++ 11's
# libstdc++ does not provide, so those standard headers are force-included (-include).
# base/FileParser.cpp / base/PlyReader.cpp / base/STLReader.cpp need C++23 library features
# (std::unreachable, std::format) absent here and are not built (see ref_harness.cpp).
set -euo pipefail
REF=${REF:-/root/reference}
HERE="$(cd "$(dirname "$0")" && pwd)"
OUT="$HERE/_ref"
[ -d "$REF" ] || { echo "build_ref: $REF not present, skipping"; exit 0; }
mkdir -p "$OUT"
FLAGS="-std=gnu++20 -O2 -ffp-contract=off -mfma -mavx2 -fPIC -w -I$REF"
INC="-include optional -include algorithm -include numeric -include sstream -include iomanip -include mutex -include cstring -include limits -include atomic"
SRCS="Integrators/Integrator.cpp materials/Material.cpp math/Sampling.cpp shapes/Triangle.cpp base/Logger.cpp Image/Image.cpp"
pids=()
for s in $SRCS; do
  o="$OUT/$(basename "$s" .cpp).o"
  if [ ! -f "$o" ] || [ "$REF/$s" -nt "$o" ] || [ "$0" -nt "$o" ]; then
    g++ $FLAGS $INC -c "$REF/$s" -o "$o" &
    pids+=($!)
  fi
done
h="$OUT/ref_harness.o"
if [ ! -f "$h" ] || [ "$HERE/ref_harness.cpp" -nt "$h" ] || [ "$0" -nt "$h" ]; then
  g++ $FLAGS $INC -c "$HERE/ref_harness.cpp" -o "$h" &
  pids+=($!)
fi
for p in "${pids[@]}"; do wait "$p"; done
g++ -shared -o "$OUT/libsp_ref.so" "$OUT"/*.o -pthread
echo "build_ref: $OUT/libsp_ref.so"
