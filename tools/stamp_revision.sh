#!/bin/bash
# tools/stamp_revision.sh -- write REVISION (git HEAD + a hash of the uncommitted state: changes to tracked files and
# the contents of untracked, non-ignored files) at the repo root before a gpurun call, so GPU logs name the exact
# tree they ran on (commit messages name the stamp a committed tree was tested as).
R=$(cd "$(dirname "$0")/.." && pwd)
cd "$R"
state_hash() {   # $1 = base commit: tracked changes since it + the untracked files
  { git diff "$1" -- . ':!REVISION' ':!profiles'; git ls-files -o --exclude-standard -- . ':!REVISION' ':!profiles' | sort | while read -r f; do
      echo "== $f"; cat "$f"; done; } | sha1sum | cut -c1-12
}
head=$(git rev-parse HEAD)
if git diff --quiet HEAD -- . ':!REVISION' ':!profiles' && [ -z "$(git ls-files -o --exclude-standard -- . ':!REVISION' ':!profiles')" ]; then
  echo "$head" > REVISION
else
  echo "$head+dirty-$(state_hash HEAD)" > REVISION
fi
cat REVISION
