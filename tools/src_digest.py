"""Digest of the sources libtiflash_amd.so is built from: every *.hip / *.h under
tiflash_amd/csrc plus include/tiflash_amd.h, sorted by name, each as (name, bytes).  The Makefile
embeds it in the library's build stamp (tfg_version); __graft_entry__.smoke() recomputes it on the
tree it runs from, so a prebuilt library that does not match its sources is reported."""
import glob
import hashlib
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def src_digest(root: str = ROOT) -> str:
    csrc = os.path.join(root, "tiflash_amd", "csrc")
    names = sorted(os.path.basename(p) for p in glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")))
    h = hashlib.sha256()
    for name in names:
        with open(os.path.join(csrc, name), "rb") as f:
            data = f.read()
        h.update(name.encode() + b"\0" + len(data).to_bytes(8, "little") + data)
    with open(os.path.join(root, "include", "tiflash_amd.h"), "rb") as f:
        data = f.read()
    h.update(b"tiflash_amd.h\0" + len(data).to_bytes(8, "little") + data)
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(src_digest())
