#!/bin/bash
# Build an A/B variant of the library: densityflows.jl_amd/libdf_<name>.so with extra
# compiler flags, recompiling only the translation units named in $OBJS (default: the
# specialised-kernel units) on top of the current in-tree build.  Extra make variables
# (e.g. FLAGS_df_wide= to drop a unit's own flags) go after the flags.
#   tools/build_variant.sh <name> "<flags>" [VAR=value ...]
set -e
cd "$(dirname "$0")/../densityflows.jl_amd/csrc"
name=$1
flags=$2
shift 2
objs=${OBJS:-"df_uniform_ht1 df_uniform_ht2 df_uniform_ht4"}
make -j8 >/dev/null
rm -rf build_$name
cp -r build build_$name
for o in $objs; do rm -f build_$name/$o.o; done
make -j8 BUILD=build_$name OUT=../libdf_$name.so EXTRA="$flags" "$@" >/dev/null
echo "built densityflows.jl_amd/libdf_$name.so ($flags $*)"
