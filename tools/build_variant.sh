#!/bin/bash
# Build an A/B variant of libmvsv.so: copy csrc, apply a sed script to one
# source file, build into variants/NAME.so.
# Usage: tools/build_variant.sh NAME FILE 'sed-script'
set -e
NAME=$1; FILE=$2; SED=$3
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d /tmp/mvsv_variant.XXXX)
mkdir -p $T/mvstereovision3_amd/csrc $T/include $R/variants
cp $R/mvstereovision3_amd/csrc/* $T/mvstereovision3_amd/csrc/
cp $R/include/mvsv.h $T/include/
sed -i "$SED" $T/mvstereovision3_amd/csrc/$FILE
if cmp -s $R/mvstereovision3_amd/csrc/$FILE $T/mvstereovision3_amd/csrc/$FILE; then echo "sed changed nothing"; exit 1; fi
make -s -C $T/mvstereovision3_amd/csrc OUT=$R/variants/$NAME.so -j8 >/dev/null
rm -rf $T
echo built variants/$NAME.so
