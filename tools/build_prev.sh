#!/bin/bash
# Build variants/NAME.so from the working tree with FILE (a csrc source) as of
# git revision REV -- a same-box A/B baseline for one file's change.
# Usage: tools/build_prev.sh NAME REV FILE
set -e
NAME=$1; REV=$2; FILE=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/mvsv_prev.XXXX)
mkdir -p $T/mvstereovision3_amd/csrc $T/include $R/variants
cp $R/mvstereovision3_amd/csrc/* $T/mvstereovision3_amd/csrc/
cp $R/include/mvsv.h $T/include/
git -C $R show $REV:mvstereovision3_amd/csrc/$FILE > $T/mvstereovision3_amd/csrc/$FILE
make -s -C $T/mvstereovision3_amd/csrc OUT=$R/variants/$NAME.so OBJDIR=$T/obj -j8 >/dev/null
rm -rf $T
echo built variants/$NAME.so
