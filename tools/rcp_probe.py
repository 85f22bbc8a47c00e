import sys, numpy as np
sys.path[:0]=['wc-path-tracer_amd']
import wcpt
ctx = wcpt.Context(0)
hi = np.arange(65536, dtype=np.uint32)
for fn in (10, 11):
    bad = ctx.selftest(fn, hi)
    nz = np.nonzero(bad)[0]
    print(fn, int(bad.sum()), "bad high halves:", [hex(int(h)) for h in nz[:20]], "...", [hex(int(h)) for h in nz[-10:]])
