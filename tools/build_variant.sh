#!/bin/bash
# build_variant.sh NAME "EXTRA FLAGS" -> tools/variants/libmigym_NAME.so
# (own object directory: the in-tree library and its objects are left alone)
set -e
cd "$(dirname "$0")/../test_isaacgym_amd/csrc"
mkdir -p ../../tools/variants
rm -rf build_v_$1
make -s -j8 OBJDIR=build_v_$1 EXTRA="$2" OUT=../../tools/variants/libmigym_$1.so
rm -rf build_v_$1
