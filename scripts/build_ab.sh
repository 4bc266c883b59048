#!/bin/bash
# Build the HIP library of another git revision as an A/B timing variant: mat_dcml_amd/_lib/libmatdcml_ab_<name>.so
#   scripts/build_ab.sh <rev> <name>        (e.g. scripts/build_ab.sh HEAD~1 base)
set -e
rev=$1; name=$2
wt=/tmp/mdl_ab_$name
rm -rf $wt; git worktree prune
git worktree add -f --detach $wt $rev > /dev/null
( cd $wt && MAT_DCML_LIBNAME=libmatdcml_ab_$name.so python mat_dcml_amd/csrc/build.py > /dev/null )
cp $wt/mat_dcml_amd/_lib/libmatdcml_ab_$name.so mat_dcml_amd/_lib/
git worktree remove --force $wt
echo "built mat_dcml_amd/_lib/libmatdcml_ab_$name.so from $(git rev-parse --short $rev)"
