#!/bin/bash
# Build libmvsv.so from a git revision (or the working tree with REF=WT) into variants/NAME.so.
# Usage: tools/build_ref.sh NAME REF [extra hipcc flags]
set -e
NAME=$1; REF=$2; EXTRA=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/mvsv_ref.XXXX)
mkdir -p $T/mvstereovision3_amd/csrc $T/include $R/variants
if [ "$REF" = "WT" ]; then
  cp $R/mvstereovision3_amd/csrc/* $T/mvstereovision3_amd/csrc/; cp $R/include/mvsv.h $T/include/
else
  git -C $R archive $REF mvstereovision3_amd/csrc include/mvsv.h | tar -x -C $T
fi
[ -n "$EXTRA" ] && sed -i "s|^FLAGS   := |FLAGS   := $EXTRA |" $T/mvstereovision3_amd/csrc/Makefile
make -s -C $T/mvstereovision3_amd/csrc OUT=$R/variants/$NAME.so -j8 >/dev/null 2>&1
rm -rf $T
echo built variants/$NAME.so
