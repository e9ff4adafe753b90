#!/bin/bash
# Build the kernels object with extra compiler flags into path_planning_pkg_amd/lib_<tag>/, reusing
# the main build's other objects (round-6 compiler-flag sweep; tools/ab_bench.sh compares them):
#   tools/flag_variants.sh <tag> "<extra flags>"
set -e
T=$1; X=$2
R=$(cd "$(dirname "$0")/.." && pwd)
D=$R/path_planning_pkg_amd/lib_$T
mkdir -p $D
for o in hastar_units_k hastar_relaxed hastar_capi hastar_units hastar_f64_k hastar_f64; do cp -p $R/path_planning_pkg_amd/lib/$o.o $D/; done
rm -f $D/hastar_kernels.o $D/libhastar_amd.so
make -s -C $R/path_planning_pkg_amd/csrc OUTDIR=$D EXTRA="$X" > $D/build.log 2>&1
bash $R/tools/kernel_regs.sh $D/hastar_kernels.o | grep search >> $D/build.log
echo "$T: $X" >> $D/build.log
