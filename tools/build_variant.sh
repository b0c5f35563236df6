#!/bin/bash
# Build an A/B variant of the native library: regenerate fs_sparse_asm.inc
# with the generator options given as environment assignments, build into
# fastselect_amd/_variants/libfastselect_amd_<name>.so (loaded with
# FS_LIB_VARIANT=<name>), then restore the default .inc.
#   tools/build_variant.sh <name> [VAR=value ...] [-- extra HIPFLAGS]
set -euo pipefail
cd "$(dirname "$0")/.."
NAME=$1; shift
ENVS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do ENVS+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
EXTRA="$*"
env "${ENVS[@]}" python3 tools/gen_sparse_asm.py > /dev/null
mkdir -p fastselect_amd/_variants
make -s -j8 -C fastselect_amd/csrc BUILD=../_vbuild/$NAME OUT=../_variants/libfastselect_amd_$NAME.so \
    HIPFLAGS="-O3 -fPIC -std=c++17 --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -Wall -fvisibility=hidden $EXTRA"
python3 tools/gen_sparse_asm.py > /dev/null
echo "built fastselect_amd/_variants/libfastselect_amd_$NAME.so"
