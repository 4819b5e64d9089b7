#!/bin/bash
# Build the library of a git revision (default HEAD) into tools/libfiode_base.so for an A/B against
# the working tree (tools/gpu_lib_ab.sh).  Not product code.
set -eu
REV=${1:-HEAD}
R=$(git rev-parse --show-toplevel)
T=$(mktemp -d /tmp/fiode_base.XXXX)
git -C "$R" archive "$REV" fi-ode_amd/csrc include | tar -x -C "$T"
make -C "$T/fi-ode_amd/csrc" -j8 OUT="$R/tools/libfiode_base.so" OBJDIR="$T/build" > /dev/null
rm -rf "$T"
echo "tools/libfiode_base.so <- $REV"
