import sys, time, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import roaringbitmap_amd as rb
import _gen, _oracle as O
from _fmt import encode
rng = np.random.default_rng(7)
k1, v1 = _gen.container(rng, "a_small")
k2, v2 = _gen.container(rng, "a_small")
a = rb.RoaringBitmap(encode([(3, k1, v1)]))
b = rb.RoaringBitmap(encode([(3, k2, v2)]))
for op in ["and", "or", "xor", "andnot"]:
    t = time.time()
    r = rb.RoaringBitmap._pair(op, a, b)
    print(op, round(time.time() - t, 4), r.serialize() == O.pairwise(op, a.serialize(), b.serialize()), flush=True)
e = rb.Engine(0)
ia = e.load([a]); ib = e.load([b])
e.profile(4)
for op in ["and", "or"]:
    e.pairwise(op, ia, ib)
e.sync()
print(e.profile_read(), flush=True)
