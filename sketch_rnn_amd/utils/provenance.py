"""Identity of the source tree a run used, recorded by the run itself
(bench.py, scripts/converge.py) instead of a label taken from the
environment.

* ``source_sha16``: sha256 over every tracked-type source file of the tree
  (``csrc/``, ``sketch_rnn_amd/``, ``scripts/``, ``bench.py``), in path
  order -- recomputable from any checkout, so a record can be matched to the
  commit whose tree hashes the same (``python -m
  sketch_rnn_amd.utils.provenance`` prints it);
* ``git_head`` / ``git_dirty``: from ``git`` when the tree is a checkout; on
  a GPU box (a snapshot without ``.git``) from ``TREE_COMMIT``, which
  ``scripts/snapshot_commit.sh`` writes before the tree is sent, and
  ``None`` when neither exists.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
from typing import Dict, Optional

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_EXT = (".py", ".hip", ".h", ".cpp", ".sh")


def source_files():
    out = []
    for top in ("csrc", "sketch_rnn_amd", "scripts"):
        for dp, dns, fns in os.walk(os.path.join(ROOT, top)):
            dns[:] = sorted(d for d in dns if d != "__pycache__")
            out += [os.path.join(dp, f) for f in sorted(fns) if f.endswith(_EXT)]
    out.append(os.path.join(ROOT, "bench.py"))
    return sorted(out)


def source_sha16() -> str:
    h = hashlib.sha256()
    for f in source_files():
        h.update(os.path.relpath(f, ROOT).encode())
        with open(f, "rb") as fh:
            h.update(hashlib.sha256(fh.read()).digest())
    return h.hexdigest()[:16]


def _git(*args) -> Optional[str]:
    try:
        return subprocess.run(["git", "-C", ROOT] + list(args), capture_output=True, text=True, timeout=10,
                              check=True).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return None


def tree_identity() -> Dict[str, object]:
    head = _git("rev-parse", "HEAD") if os.path.isdir(os.path.join(ROOT, ".git")) else None
    if head:
        dirty = bool(_git("status", "--porcelain", "--untracked-files=no"))
        src = "git"
    else:
        head, dirty, src = None, None, None
        path = os.path.join(ROOT, "TREE_COMMIT")
        if os.path.exists(path):
            with open(path) as f:
                parts = f.read().split()
            if parts:
                head, dirty, src = parts[0], (len(parts) > 1 and parts[1] == "dirty"), "TREE_COMMIT"
    return {"git_head": head, "git_dirty": dirty, "git_source": src, "source_sha16": source_sha16()}


if __name__ == "__main__":
    import json
    print(json.dumps(tree_identity()))
