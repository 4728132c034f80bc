#!/bin/bash
# Build a reference tree of an earlier revision for same-box A/B timing:
#   bash scripts/ab_build.sh <rev>   -> build/ab/A (a git worktree of <rev>, extension built)
# then on the GPU box:  STAGES=ab bash scripts/gpu_r05.sh  (alternates A and the working tree)
set -eu
rev=${1:?revision}
rm -rf build/ab/A
git worktree prune
mkdir -p build/ab
git worktree add --detach build/ab/A "$rev" > /dev/null
(cd build/ab/A && python -c "from distributed_amd import _build; _build.build()" > /dev/null)
echo "A = $(git -C build/ab/A log --oneline -1)"
