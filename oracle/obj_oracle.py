"""ORACLE (test infrastructure only) — pure-Python restatement of parse_obj_file (src/ModelLoader.jai:60-141).

Small inputs only (the reference's asset OBJs are < 70 KB). Float parsing: the reference uses Jai's
string_to_float (the Jai Basic module is not in the container, version unpinned); this restatement parses
with Python float() and rounds to binary32, which equals correctly rounded strtof for the short decimals
of OBJ files. Face indices follow :103-136: 1-based, (v, vt, vn) key de-duplication in first-seen order,
fan triangulation.
"""
from __future__ import annotations

import numpy as np


def _to_float(tok: str) -> float:
    # leading float of the token, 0 when nothing parses (Jai string_to_float returns 0 on failure)
    for end in range(len(tok), 0, -1):
        try:
            return float(tok[:end])
        except ValueError:
            continue
    return 0.0


def _to_int(tok: str) -> int:
    i, neg = 0, False
    if i < len(tok) and tok[i] in "+-":
        neg, i = tok[i] == "-", i + 1
    j = i
    while j < len(tok) and tok[j].isdigit():
        j += 1
    if j == i:
        return 0
    v = int(tok[i:j])
    return -v if neg else v


def parse_obj(text: str):
    """Returns (positions float32 [V,3], indices uint32 [I])."""
    positions, out_pos, out_idx = [], [], []
    vmap = {}
    for line in text.split("\n"):
        t = line.strip(" \t\r\n\v\f")
        if not t or t[0] == "#":
            continue
        tokens = t.split(" ")
        cmd = tokens[0]
        if cmd == "v" and len(tokens) >= 4:
            positions.append(tuple(np.float32(_to_float(x)) for x in tokens[1:4]))
        elif cmd == "f" and len(tokens) >= 4:
            face = []
            for tok in tokens[1:]:
                parts = tok.split("/")
                key = [-1, -1, -1]
                for k in range(3):
                    if len(parts) > k and parts[k]:
                        key[k] = _to_int(parts[k]) - 1
                key = tuple(key)
                if key not in vmap:
                    p = positions[key[0]] if 0 <= key[0] < len(positions) else (0.0, 0.0, 0.0)
                    vmap[key] = len(out_pos)
                    out_pos.append(p)
                face.append(vmap[key])
            for i in range(1, len(face) - 1):
                out_idx += [face[0], face[i], face[i + 1]]
    return (np.array(out_pos, np.float32).reshape(-1, 3), np.array(out_idx, np.uint32))
