#!/bin/bash
# tools/stamp_revision.sh -- write REVISION (git HEAD + a hash of uncommitted changes to tracked files)
# at the repo root before a gpurun call, so GPU logs name the exact tree they ran on.
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
head=$(git rev-parse HEAD)
if git diff --quiet HEAD -- . ':!REVISION'; then
  echo "$head" > REVISION
else
  echo "$head+dirty-$(git diff HEAD -- . ':!REVISION' | sha1sum | cut -c1-12)" > REVISION
fi
cat REVISION
