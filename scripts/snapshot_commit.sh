#!/bin/bash
# Write TREE_COMMIT (HEAD + clean/dirty) at the repo root before a tree is
# sent to a GPU box that has no .git: sketch_rnn_amd/utils/provenance.py
# reads it there. Usage: scripts/snapshot_commit.sh && gpurun -- ...
cd "$(dirname "$0")/.." || exit 1
head=$(git rev-parse HEAD) || exit 1
if [ -n "$(git status --porcelain --untracked-files=no)" ]; then state=dirty; else state=clean; fi
echo "$head $state" > TREE_COMMIT
