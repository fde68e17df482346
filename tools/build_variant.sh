#!/bin/bash
# Experiment builds: libh12env_<name>.so next to the in-tree library, same flags plus the given -D options
# (bench.py / tests pick one with H12ENV_LIB=<path>).  Usage: bash tools/build_variant.sh <name> -DFOO=1 ...
set -e
name=$1
shift
cd "$(dirname "$0")/.."
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -Xarch_device -ffinite-math-only \
  -Xarch_device -fno-signed-zeros -fPIC -shared -Wall -Wno-unused-function "$@" \
  -o h1v2-isaac_amd/h12env/libh12env_$name.so h1v2-isaac_amd/csrc/h12env.hip
