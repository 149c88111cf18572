"""``python -m sketch_rnn_amd.cli.preprocess`` -- dataset preparation.

* ``svg DIR OUT.npz``: SVG corpus -> reference stroke-4 cache (R4; the
  reference's ``data/<name>.cpkl`` step, ``utils.py:124-217``, without pickle);
* ``quickdraw OUT.skpack.npz A.npz [B.npz ...] --allow-pickle``: public
  QuickDraw files (object arrays; only for files you trust) -> sketch pack,
  one class label per input file;
* ``synthetic OUT.skpack.npz --n N``: synthetic corpus in pack format.
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    p = argparse.ArgumentParser()
    sub = p.add_subparsers(dest="cmd", required=True)
    s = sub.add_parser("svg")
    s.add_argument("data_dir")
    s.add_argument("out")
    s.add_argument("--verbose", action="store_true")
    q = sub.add_parser("quickdraw")
    q.add_argument("out")
    q.add_argument("inputs", nargs="+")
    q.add_argument("--allow-pickle", action="store_true")
    y = sub.add_parser("synthetic")
    y.add_argument("out")
    y.add_argument("--n", type=int, default=10000)
    y.add_argument("--classes", type=int, default=1)
    y.add_argument("--max_len", type=int, default=250)
    y.add_argument("--seed", type=int, default=0)
    a = p.parse_args(argv)
    if a.cmd == "svg":
        from ..data.preprocess import preprocess
        sk, _ = preprocess(a.data_dir, a.out, verbose=a.verbose)
        print("wrote %d sketches to %s" % (len(sk), a.out))
    elif a.cmd == "quickdraw":
        from ..data.quickdraw import convert_to_pack
        convert_to_pack(a.inputs, a.out, allow_pickle=a.allow_pickle)
        print("wrote %s" % a.out)
    else:
        from ..data.quickdraw import save_pack
        from ..data.synthetic import synthetic_corpus
        s, l = synthetic_corpus(a.n, seed=a.seed, max_len=a.max_len, n_classes=a.classes)
        k = max(a.n // 10, 1)
        save_pack(a.out, {"train": (s[2 * k:], l[2 * k:]), "valid": (s[:k], l[:k]), "test": (s[k:2 * k], l[k:2 * k])})
        print("wrote %s" % a.out)
    return 0


if __name__ == "__main__":
    sys.exit(main())
