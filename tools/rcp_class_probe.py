"""Exhaustive check of the result-validated reciprocal (pt_device.h rcp_exact, rcp2_exact) on the device: selftest fn 12 counts
mismatches against the IEEE quotient over all 2^32 inputs, fn 13 counts the inputs that take the general division."""
import sys
import numpy as np
sys.path[:0] = ['wc-path-tracer_amd']
import wcpt
ctx = wcpt.Context(0)
hi = np.arange(65536, dtype=np.uint32)
bad = ctx.selftest(12, hi)
slow = ctx.selftest(13, hi)
nz = np.nonzero(bad)[0]
print("rcp_exact + rcp2_exact mismatches over 2^32 inputs:", int(bad.sum()), [hex(int(h)) for h in nz[:16]])
print("inputs on the general division:", int(slow.astype(np.uint64).sum()))
