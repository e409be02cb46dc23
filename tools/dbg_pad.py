import sys, importlib
sys.path[:0] = ['.', 'tests']
import numpy as np, torch
import mvxtest as T
mvx = importlib.import_module("mvapich-cce_amd")
from oracle import oracle as O
import hashlib
print("lib md5", hashlib.md5(open(mvx.LIB_HIP,'rb').read()).hexdigest())
for op in (110, 111):
    n = 4099
    a, b = T.rand_vec(18, n, 11), T.rand_vec(18, n, 12)
    da, db = T.to_dev(a), T.to_dev(b)
    rc = mvx.op_apply(op, 18, da, db, n)
    got = T.from_dev(db).view(np.uint8).reshape(n, 16)
    ref = b.copy(); O.op(op, 18, a.view(np.uint8), ref.view(np.uint8), n)
    refb = ref.view(np.uint8).reshape(n, 16)
    print(op, rc, "got pad nonzero:", int((got[:, 12:] != 0).any(1).sum()), "ref pad nonzero:", int((refb[:, 12:] != 0).any(1).sum()),
          "in pad nonzero", int((a.view(np.uint8).reshape(n,16)[:,12:]!=0).any(1).sum()), "diff rows", int((got != refb).any(1).sum()))
    bad = np.nonzero((got != refb).any(1))[0][:3]
    for r in bad:
        print(r, got[r], refb[r], a.view(np.uint8).reshape(n,16)[r], b.view(np.uint8).reshape(n,16)[r])
