#!/bin/bash
# A/B diagnostics: build libkpsim from the sources of a git commit into tools/ab/<name>.so (sources and objects under
# /tmp), e.g. tools/build_commit.sh r05 94acf4b — to time a round's library against the working tree's on one box.
set -euo pipefail
NAME=$1; REV=$2; shift 2
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=/tmp/kpcommit_$NAME
rm -rf "$SRC" && mkdir -p "$SRC" "$ROOT/tools/ab"
git -C "$ROOT" archive "$REV" karpenter-provider-aws_amd/csrc karpenter-provider-aws_amd/Makefile include | tar -x -C "$SRC"
make -s -j8 -C "$SRC/karpenter-provider-aws_amd" "$@" lib/libkpsim.so
cp "$SRC/karpenter-provider-aws_amd/lib/libkpsim.so" "$ROOT/tools/ab/$NAME.so"
echo "built tools/ab/$NAME.so from $REV"
