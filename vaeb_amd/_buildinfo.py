"""The source-hash stamp of libvaeb_hip.so (written by __graft_entry__.build(), checked by
vaeb_amd._lib.load()): a prebuilt library whose stamp does not match the sources next to it
is refused, so a stale .so can never run silently (on the GPU box the driver runs the
pushed, prebuilt library without building)."""
import hashlib
import os

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wno-unused-result", "-Wno-unused-value"]


def source_hash() -> str:
    """sha256 over the library's sources (vaeb_amd/csrc/*, include/*.h) and the build flags."""
    h = hashlib.sha256(" ".join(FLAGS).encode())
    for d in (CSRC, INCLUDE):
        for f in sorted(os.listdir(d)):
            if f.endswith((".hip", ".hpp", ".inc", ".h")):
                h.update(f.encode())
                with open(os.path.join(d, f), "rb") as fh:
                    h.update(fh.read())
    return h.hexdigest()


def stamp_path(lib_path: str) -> str:
    return lib_path + ".srchash"


def check_stamp(lib_path: str):
    """None when lib_path's stamp matches the sources, else the reason it does not."""
    if not os.path.isdir(CSRC):
        return None   # an installed copy without sources: nothing to compare
    sp = stamp_path(lib_path)
    if not os.path.exists(sp):
        return f"{sp} is missing (the library was not built by __graft_entry__.build())"
    have = open(sp).read().strip()
    want = source_hash()
    if have != want:
        return f"{os.path.basename(lib_path)} was built from other sources (stamp {have[:12]}, sources {want[:12]})"
    return None
