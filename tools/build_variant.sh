#!/bin/bash
# build_variant.sh NAME "EXTRA FLAGS" -> tools/variants/libmigym_NAME.so
set -e
cd "$(dirname "$0")/../test_isaacgym_amd/csrc"
mkdir -p ../../tools/variants
make -s clean >/dev/null 2>&1 || true
make -s EXTRA="$2" OUT=../../tools/variants/libmigym_$1.so
make -s clean >/dev/null 2>&1 || true
make -s
