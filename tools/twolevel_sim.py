"""CPU estimate of the dependent round trips a two-level child-pair fetch would save in the wavefront trace.

Walks rays through a scene's midpoint BVH the way wf_trace does (near child entered directly, far child pushed unless
it fails or its entry is beyond rec.t, popped entries culled against rec.t; pathTracer.comp:150-200) and counts the
dependent memory round trips per ray: one per interior visit (the child pair) and one per triangle test (the record).
The two-level variant also loads, with each child pair, the child pair of the child predicted to be near (the lower
half along the node's split axis when the ray's direction along it is positive, the upper half otherwise); when that
child is the one entered and it is interior, its interior step needs no fetch.

    python tools/twolevel_sim.py [--scene atrium] [--w 160] [--h 90] [--bounces 2]
Approximate rays (float64, primary rays plus uniform hemisphere bounces): an estimate, not a parity tool.
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "wc-path-tracer_amd"))
from wcpt import scene as wscene  # noqa: E402


def box(o, inv, bmin, bmax):
    with np.errstate(invalid="ignore", over="ignore"):
        tb = (bmin - o) * inv
        tt = (bmax - o) * inv
    tmin = np.minimum(tt, tb)
    tmax = np.maximum(tt, tb)
    return max(tmin[0], tmin[1], tmin[2]), min(tmax[0], tmax[1], tmax[2])


def tri(o, d, a, b, c):
    e1, e2 = b - a, c - a
    p = np.cross(d, e2)
    det = e1 @ p
    if det == 0.0:
        return -1.0
    inv = 1.0 / det
    s = o - a
    u = (s @ p) * inv
    q = np.cross(s, e1)
    v = (d @ q) * inv
    t = (e2 @ q) * inv
    return t if (t > 0 and u >= 0 and v >= 0 and u + v <= 1) else -1.0


def walk(o, d, N, V, I, axis, two_level):
    inv = 1.0 / np.where(d == 0.0, 1e-30, d)
    rt = np.inf
    rts = 0
    hitp = None
    c0, c1 = box(o, inv, N["min"][0], N["max"][0])
    if c0 > c1 or c1 < 0:
        return rts, rt
    stack = []
    cur = 0
    pre = False          # cur's child pair is already in registers (two-level hit)
    while True:
        if cur is None:
            if not stack:
                break
            ni, t0 = stack.pop()
            if t0 > rt:
                continue
            cur, pre = ni, False
        cnt = int(N["triangleCount"][cur])
        first = int(N["leftNodeOrTriangleIndex"][cur])
        if cnt > 0:
            for k in range(first, first + cnt, 3):
                rts += 1
                tt = tri(o, d, V[I[k]], V[I[k + 1]], V[I[k + 2]])
                if tt != -1.0 and tt < rt:
                    rt = tt
            cur = None
            continue
        if not pre:
            rts += 1
        L, R = first, first + 1
        l0, l1 = box(o, inv, N["min"][L], N["max"][L])
        r0, r1 = box(o, inv, N["min"][R], N["max"][R])
        ld = l0 if l0 > 0 else l1
        rd = r0 if r0 > 0 else r1
        lf = ld < rd
        passL = not (l0 > l1 or l1 < 0)
        passR = not (r0 > r1 or r1 < 0)
        near, far = (L, R) if lf else (R, L)
        pn, pf = (passL, passR) if lf else (passR, passL)
        n0, f0 = (l0, r0) if lf else (r0, l0)
        if pf and not (f0 > rt):
            stack.append((far, f0))
        if pn and not (n0 > rt):
            pred = L if d[axis[cur]] > 0 else R
            pre = two_level and near == pred and int(N["triangleCount"][near]) == 0
            cur = near
        else:
            cur = None
    return rts, rt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="atrium")
    ap.add_argument("--w", type=int, default=160)
    ap.add_argument("--h", type=int, default=90)
    ap.add_argument("--bounces", type=int, default=2)
    args = ap.parse_args()
    s = wscene.generate(args.scene)
    m = s.meshes[0]
    N, V, I = m.nodes, m.positions.astype(np.float64), m.indices.astype(np.int64)
    ext = N["max"] - N["min"]
    axis = np.where(ext[:, 1] > ext[:, 0], 1, 0)
    axis = np.where(ext[:, 2] > ext[np.arange(len(N)), axis], 2, axis)
    sd = s.scene_data(args.w, args.h)
    ip = np.asarray(sd["inverseProjection"], np.float64).reshape(4, 4)
    iv = np.asarray(sd["inverseView"], np.float64).reshape(4, 4)
    pos = np.asarray(sd["position"], np.float64)
    rng = np.random.default_rng(1)
    tot = {False: 0, True: 0}
    rays = 0
    for y in range(args.h):
        for x in range(args.w):
            cx = (x + 0.5) / args.w * 2 - 1
            cy = (1 - (y + 0.5) / args.h) * 2 - 1
            tg = np.array([cx, cy, 1.0, 1.0]) @ ip
            dv = tg[:3] / tg[3]
            dv /= np.linalg.norm(dv)
            d = (np.array([dv[0], dv[1], dv[2], 0.0]) @ iv)[:3]
            d /= np.linalg.norm(d)
            o = pos.copy()
            for b in range(args.bounces + 1):
                r0, t = walk(o, d, N, V, I, axis, False)
                r1, _ = walk(o, d, N, V, I, axis, True)
                tot[False] += r0
                tot[True] += r1
                rays += 1
                if not np.isfinite(t):
                    break
                o = o + t * d
                nd = rng.normal(size=3)
                nd /= np.linalg.norm(nd)
                if nd @ d > 0:
                    nd = -nd
                d = nd
                o = o + 1e-4 * d
    print(f"{rays} rays: round trips per ray {tot[False] / rays:.2f} -> {tot[True] / rays:.2f} "
          f"({1 - tot[True] / tot[False]:.1%} fewer)")


if __name__ == "__main__":
    main()
