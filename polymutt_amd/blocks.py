"""Reader for the dense indexed site-block format (.pmb, polymutt_amd/host/blocks.h).

`polymutt --glf2blocks OUT.pmb -p PED -d DAT -g GIF` writes one; `polymutt --in_blocks FILE` analyses it.
This module gives random access to its blocks -- e.g. one shard of a section per GPU rank -- as the arrays
pm_engine_run takes (pl [n][n_person][10] u8, dm [n][n_person] u32 = depth | mapQ << 24, ref [n] u8).
"""
import struct

import numpy as np

_ENTRY = struct.Struct("<IIiiQ")


def read_header(path):
    with open(path, "rb") as fh:
        magic, n_person, block_sites, _ = struct.unpack("<4sIII", fh.read(16))
    if magic != b"PMB1":
        raise ValueError(f"{path}: not a polymutt block file")
    return {"n_person": n_person, "block_sites": block_sites}


def read_index(path):
    """[{section, n, first_pos, last_pos, offset}] from the file's trailing index."""
    with open(path, "rb") as fh:
        fh.seek(-12, 2)
        at, end = struct.unpack("<Q4s", fh.read(12))
        if end != b"PMBE":
            raise ValueError(f"{path}: missing trailer")
        fh.seek(at)
        tag, nb = struct.unpack("<4sI", fh.read(8))
        if tag != b"PIDX":
            raise ValueError(f"{path}: missing index")
        raw = fh.read(nb * _ENTRY.size)
    return [dict(zip(("section", "n", "first_pos", "last_pos", "offset"), _ENTRY.unpack_from(raw, i * _ENTRY.size)))
            for i in range(nb)]


def read_sections(path):
    """[(label, maxPosition)] in file order."""
    out = []
    with open(path, "rb") as fh:
        np_ = read_header(path)["n_person"]
        fh.seek(16)
        while True:
            tag = fh.read(4)
            if tag != b"SECT":
                return out
            mp, ln = struct.unpack("<iI", fh.read(8))
            out.append((fh.read(ln).decode(), mp))
            while True:
                t = fh.read(4)
                if t == b"SEND":
                    fh.read(8)
                    break
                n, = struct.unpack("<I", fh.read(4))
                fh.seek(n * (4 + 1 + np_ * 14), 1)


def read_block(path, entry, n_person=None):
    """(pos [n] 0-based i32, ref [n] u8, pl [n][n_person][10] u8, dm [n][n_person] u32) of one index entry."""
    if n_person is None:
        n_person = read_header(path)["n_person"]
    with open(path, "rb") as fh:
        fh.seek(entry["offset"])
        tag, n = struct.unpack("<4sI", fh.read(8))
        if tag != b"BLK1" or n != entry["n"]:
            raise ValueError(f"{path}: index entry does not point at a block")
        pos = np.frombuffer(fh.read(4 * n), "<i4")
        ref = np.frombuffer(fh.read(n), np.uint8)
        pl = np.frombuffer(fh.read(n * n_person * 10), np.uint8).reshape(n, n_person, 10)
        dm = np.frombuffer(fh.read(n * n_person * 4), "<u4").reshape(n, n_person)
    return pos, ref, pl, dm
