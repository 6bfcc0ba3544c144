"""Fresh-process check: the ragged OU case's first draws (k_block_scan) as the first device work
of a process, device == oracle on the drawn paths and the returned log-likelihoods."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)
import _cases as cs
from diffusionmcmctools_amd import _lib as L

case, dev, ora, ids = cs.ragged_pair(model=cs.ou_ragged_model())
for u in (L.U, L.UPROP):
    for w in (0, 1):
        a, b = dev.download_paths(u, w), ora.download_paths(u, w)
        assert np.array_equal(a, b), (u, w)
for lid, nb in ids:
    for e in (dev, ora):
        e.loglikhd(lid, L.U, 0, nb)
    a, b = dev.get_block_state(lid, L.BLK_LL, 0, nb), ora.get_block_state(lid, L.BLK_LL, 0, nb)
    assert np.array_equal(a, b), (a, b)
print("ou fresh-process check OK")
