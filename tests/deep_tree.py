"""A hand-made BVH deeper than the reference's traversal stack (test input, no product code).

A chain of `levels` interior nodes, each with a one-triangle leaf as its left child and the next interior node as its
right child, every box the mesh's whole box. Both children always pass and tie on distance, so the reference pushes
left then right (pathTracer.comp:192-198) and pops the interior child first: the stack grows by one entry per level
and a ray that reaches the bottom has written nodeStack[levels] -- past the reference's uint nodeStack[32] (:151) for
levels > 31 -- while this implementation's 48-entry stack holds it."""
import copy

import numpy as np

import wcpt
from wcpt import scene as wscene


def deep_chain_scene(base: "wscene.HostScene", levels: int = 40, seed: int = 3) -> "wscene.HostScene":
    rng = np.random.default_rng(seed)
    ntri = levels + 1
    centres = rng.uniform(-1.5, 1.5, (ntri, 3)).astype(np.float32)
    centres[:, 2] -= 4.0
    pos = (centres[:, None, :] + rng.uniform(-0.6, 0.6, (ntri, 3, 3)).astype(np.float32)).reshape(-1, 3)
    pos = np.ascontiguousarray(pos, dtype=np.float32)
    idx = np.arange(3 * ntri, dtype=np.uint32)
    lo, hi = pos.min(axis=0), pos.max(axis=0)
    nodes = np.zeros(2 * levels + 1, dtype=wcpt._lib.NODE_DTYPE)
    # interior k at index 2k (k < levels): children 2k+1 (leaf, triangle k) and 2k+2 (interior k+1, or the last leaf)
    for k in range(levels):
        nodes[2 * k] = (lo, hi, 2 * k + 1, 0)
        nodes[2 * k + 1] = (lo, hi, 3 * k, 3)
    nodes[2 * levels] = (lo, hi, 3 * levels, 3)
    s = copy.copy(base)
    s.meshes = [wscene.HostBVH(pos, idx, nodes)]
    return s
