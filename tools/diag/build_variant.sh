#!/bin/bash
# Build libirlmx.so with extra compile flags into build/<name>/ (git-ignored; it
# travels to the GPU box with the tree).  Load it with IRLMX_LIB=build/<name>/libirlmx.so.
# usage: tools/diag/build_variant.sh NAME -DFOO=1 ...
set -e
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
name=$1; shift
mkdir -p "$ROOT/build/$name"
cd "$ROOT/irl-maxent_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -shared -fPIC -Wall -ffp-contract=off "$@" \
  -o "$ROOT/build/$name/libirlmx.so" csrc/*.hip
