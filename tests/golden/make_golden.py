"""Regenerates tests/golden/images.npz and tests/golden/kat.json from the CPU oracle (oracle/pt_oracle.c).

    python tests/golden/make_golden.py

The reference (Jai host + GLSL/Vulkan) cannot be built or run in this container, so these
images pin the oracle and the HIP path against regressions; the RNG known answers in kat.json are the
values of SURVEY.md §4, computed independently from the formulas of src/shaders/include/Random.glsl:10-32.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "wc-path-tracer_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]

import oracle  # noqa: E402
from golden_cases import CASES  # noqa: E402
from wcpt import scene as wscene  # noqa: E402


def pcg_ref(x):
    m = 0xFFFFFFFF
    st = (x * 747796405 + 2891336453) & m
    w = (((st >> ((st >> 28) + 4)) ^ st) * 277803737) & m
    return ((w >> 22) ^ w) & m


def rand_ref(state):
    w = (((state >> ((state >> 28) + 4)) ^ state) * 277803737) & 0xFFFFFFFF
    out = ((w >> 22) ^ w) & 0xFFFFFFFF
    return out, float(np.float32(out) * np.float32(2.0 ** -32))


def main():
    images = {}
    scenes = {}
    for key, (name, W, H, bounces, spp, frames) in CASES.items():
        s = scenes.setdefault(name, wscene.generate(name))
        acc = None
        for f in frames:
            acc, _ = oracle.render_scene(s, W, H, max_bounce=bounces, samples=spp, frame=f, image=acc, threads=8)
        images[key] = acc[..., :3].astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "images.npz"), **images)
    kat = {"pcg_hash": {str(x): pcg_ref(x) for x in (0, 1, 2, 719393, 2073599)}}
    st, seq = pcg_ref(0), []
    for _ in range(4):
        st, f = rand_ref(st)
        seq.append({"state": st, "float": f})
    kat["rand_from_pcg_hash_0"] = seq
    with open(os.path.join(HERE, "kat.json"), "w") as fh:
        json.dump(kat, fh, indent=1)
    print({k: v.shape for k, v in images.items()})


if __name__ == "__main__":
    main()
