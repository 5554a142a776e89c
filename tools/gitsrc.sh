#!/bin/bash
# Copy ffmpeg_distributed_amd/csrc as of a git revision into tools/_v<NAME>src (for
# tools/variants.py A/Bs against an earlier build).  Usage: bash tools/gitsrc.sh NAME [REV]
set -e
cd "$(dirname "$0")/.."
D=tools/_v$1src
rm -rf $D && mkdir -p $D
for f in $(git ls-tree --name-only ${2:-HEAD} ffmpeg_distributed_amd/csrc/); do
  git show ${2:-HEAD}:$f > $D/$(basename $f)
done
echo $D
