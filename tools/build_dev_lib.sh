#!/bin/bash
# Build the DEV_PROBES library (build container) into tools/_probe/libpt2q_dev.so from a scratch
# copy of the package sources, leaving the in-tree build alone.  bash tools/build_dev_lib.sh
set -e
R=$(cd $(dirname $0)/.. && pwd)
P=$R/snlp---tenary-post-train-quantization_amd
T=$(mktemp -d /tmp/pt2q_dev.XXXX)
mkdir -p $T/pkg $R/tools/_probe
cp -r $P/csrc $P/Makefile $T/pkg/
ln -s $R/include $T/include
make -s -C $T/pkg -j8 DEV_PROBES=1
cp $T/pkg/libpt2q.so $R/tools/_probe/libpt2q_dev.so
rm -rf $T
