#!/bin/bash
# Builds build_san/libdpwa_hip.so: the same library with its host code under UndefinedBehavior-
# Sanitizer in trap mode (a check that fails executes a trap instruction: no sanitizer runtime
# to load, so it runs inside python as is).  Device code is not instrumented.  Use it with
#   DPWA_HIP_LIB=$PWD/build_san/libdpwa_hip.so python -m pytest tests ...
# (build_san is listed in .gpurunignore: take that line out before a GPU run that loads it)
set -e
cd "$(dirname "$0")/../dpwa_amd/csrc"
mkdir -p ../../build_san
make -j8 OBJ=_obj_san LIB=../../build_san/libdpwa_hip.so \
    CXXFLAGS="-O1 -g -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=off --offload-arch=gfx950 \
-mcode-object-version=5 -Xarch_host -fsanitize=undefined -Xarch_host -fsanitize-trap=undefined \
-Xarch_host -fno-sanitize=vptr"
n=$(/opt/rocm/lib/llvm/bin/llvm-objdump -d ../../build_san/libdpwa_hip.so | grep -c "ud1\|ud2" || true)
echo "build_san/libdpwa_hip.so: $n trap sites"
