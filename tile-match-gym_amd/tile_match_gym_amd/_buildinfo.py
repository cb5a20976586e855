"""Source hash of libtmg.so: sha256 over the library's sources (csrc/, the C
header, the Makefile) in a fixed order.  The Makefile bakes it into the
library (tmg_build_info); the loader (_native.load) recomputes it from the
tree and refuses a library built from other sources.  No torch import, so the
Makefile can run this file as a script."""
from __future__ import annotations

import glob
import hashlib
import os

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))      # tile-match-gym_amd/


def source_files(pkg_root: str = PKG_ROOT):
    """(name, path) of every file the library is built from, sorted by name."""
    files = []
    for pat in ("*.hip", "*.h"):
        for p in glob.glob(os.path.join(pkg_root, "csrc", pat)):
            files.append(("csrc/" + os.path.basename(p), p))
    files.append(("include/tmg.h", os.path.join(pkg_root, "..", "include", "tmg.h")))
    files.append(("Makefile", os.path.join(pkg_root, "Makefile")))
    return sorted(files)


def source_hash(pkg_root: str = PKG_ROOT):
    """Hex sha256 of the sources, or None when they are not all present."""
    h = hashlib.sha256()
    for name, path in source_files(pkg_root):
        if not os.path.exists(path):
            return None
        h.update(name.encode() + b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    print(source_hash())
