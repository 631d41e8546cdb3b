#!/bin/bash
# build_variant_one.sh NAME SOURCE "EXTRA FLAGS" [REPLACES] -> tools/variants/libmigym_NAME.so
# (REPLACES: the in-tree source whose object SOURCE stands in for, when SOURCE is
# a modified copy, e.g. mg_env_try.hip for mg_env.hip)
# One source recompiled with EXTRA FLAGS, linked with the in-tree build's other
# objects (the in-tree build must be current): seconds instead of a full rebuild.
set -e
cd "$(dirname "$0")/../test_isaacgym_amd/csrc"
make -s
mkdir -p ../../tools/variants build_var
/opt/rocm/bin/hipcc $3 -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
    -mcode-object-version=5 -Wall -Wno-unused-result -I../../include -x hip -c "$2" -o build_var/$1.o
objs=$(ls build/*.o | grep -v "/${4:-$2}.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/variants/libmigym_$1.so build_var/$1.o $objs
echo built tools/variants/libmigym_$1.so
