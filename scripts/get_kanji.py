#!/usr/bin/env python3
"""Fetch and unpack the KanjiVG corpus the reference trains on (R19,
reference get_kanji.sh): ``data/kanji/*.svg``, with the one file the
reference rejects (``05747-Kaisho.svg``) moved to ``data/rejects/``.

    python scripts/get_kanji.py                 # download (needs network)
    python scripts/get_kanji.py --zip FILE.zip  # use an already downloaded archive

Then: ``python -m sketch_rnn_amd.cli.train --dataset_name kanji``.
"""
from __future__ import annotations

import argparse
import os
import shutil
import sys
import urllib.request
import zipfile

URL = "https://github.com/KanjiVG/kanjivg/releases/download/r20150615-2/kanjivg-20150615-2-all.zip"
REJECTS = ("05747-Kaisho.svg",)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--data_dir", default="data")
    ap.add_argument("--zip", default=None, help="local copy of the KanjiVG release archive")
    a = ap.parse_args(argv)
    os.makedirs(a.data_dir, exist_ok=True)
    path = a.zip
    if path is None:
        path = os.path.join(a.data_dir, os.path.basename(URL))
        if not os.path.exists(path):
            print("downloading", URL)
            try:
                urllib.request.urlretrieve(URL, path)
            except OSError as e:
                print("download failed (%s); pass --zip with a local copy" % e, file=sys.stderr)
                return 1
    with zipfile.ZipFile(path) as z:
        for m in z.infolist():
            # the archive's members live under kanji/; refuse anything escaping data_dir
            dest = os.path.realpath(os.path.join(a.data_dir, m.filename))
            if not dest.startswith(os.path.realpath(a.data_dir) + os.sep):
                raise ValueError("unsafe path in archive: %s" % m.filename)
        z.extractall(a.data_dir)
    rej = os.path.join(a.data_dir, "rejects")
    os.makedirs(rej, exist_ok=True)
    for name in REJECTS:
        src = os.path.join(a.data_dir, "kanji", name)
        if os.path.exists(src):
            shutil.move(src, os.path.join(rej, name))
    n = len([f for f in os.listdir(os.path.join(a.data_dir, "kanji")) if f.endswith(".svg")])
    print("%d SVG files in %s" % (n, os.path.join(a.data_dir, "kanji")))
    return 0


if __name__ == "__main__":
    sys.exit(main())
