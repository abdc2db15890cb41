"""The served-ranking parity rule shared by the trained-
ranking GPU tests: top-k positions whose items cannot trade places under the
stated score tolerances must match the oracle exactly."""
import numpy as np


def decided_positions(o, t, k):
    """o, t: oracle scores and tolerances of every candidate, in candidate
    order. Returns (order, decided): the oracle's stable descending order
    (Python's sorted(reverse=True)) and, for its first k positions, whether
    each is decided under the tolerances."""
    o = np.asarray(o, np.float64)
    t = np.asarray(t, np.float64)
    order = np.array(sorted(range(len(o)), key=lambda j: o[j], reverse=True), dtype=np.int64)
    os_, ts = o[order], t[order]
    hi = os_ + ts
    lo = os_ - ts
    # max over later positions of (o + t); min over earlier positions of (o - t)
    later_max = np.maximum.accumulate(hi[::-1])[::-1]
    later_max = np.concatenate([later_max[1:], [-np.inf]])
    earlier_min = np.minimum.accumulate(lo)
    earlier_min = np.concatenate([[np.inf], earlier_min[:-1]])
    dec = (lo > later_max) & (hi < earlier_min)
    return order, dec[:k]


def check_served(served_ids, cand_ids, o, t, k):
    """served_ids: the GPU path's top-k item ids. Returns True if every top-k
    position of this user was decided; asserts the decided ones."""
    order, dec = decided_positions(o, t, k)
    want = [cand_ids[j] for j in order[:k]]
    assert len(served_ids) == min(k, len(cand_ids))
    for j in range(len(served_ids)):
        if dec[j]:
            assert served_ids[j] == want[j], (j, served_ids, want, dec)
    # the top-k SET is decided when the boundary between k-1 and k is
    if len(o) > k and dec[k - 1]:
        assert set(served_ids) == set(want)
    return bool(dec.all())
