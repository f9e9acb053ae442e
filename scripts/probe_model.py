#!/usr/bin/env python3
"""Model of the table's probe round trips (linear probing, reads of aligned
S-slot groups), per probe and per WAVE: a wave's probe loop runs until its
last lane's key is settled, so its cost is the max over the ~128 probes of
its lanes (two seeds each).

    python scripts/probe_model.py

Homes anywhere in a group (align 1) vs homes at the start of a group of 4
(align 4) vs buckets of 8 read whole (S = 8), at the load factors of C2 / C4
(0.116), C4 with the HyperLogLog sizing (0.68) and C5 (0.48).
"""
import numpy as np


def steps(alpha, align, S=4, cap=1 << 20, seed=0):
    """Round trips of successful and unsuccessful searches."""
    rng = np.random.default_rng(seed)
    n = int(alpha * cap)
    homes = rng.integers(0, cap // align, n) * align
    occ = np.zeros(cap, bool)
    pos = np.empty(n, np.int64)
    for i, h in enumerate(homes):
        p = h
        while occ[p]:
            p = (p + 1) % cap
        occ[p] = True
        pos[i] = p
    succ = ((pos // S - homes // S) % (cap // S)) + 1
    qh = rng.integers(0, cap // align, 200_000) * align
    empty = np.where(~occ)[0]
    j = np.searchsorted(empty, qh)
    first_empty = np.where(j < len(empty), empty[np.minimum(j, len(empty) - 1)], empty[0] + cap)
    return succ, (first_empty // S - qh // S) + 1


def main():
    rng = np.random.default_rng(5)
    for alpha in (0.116, 0.33, 0.48, 0.68):
        for align, S in ((1, 4), (4, 4), (8, 8)):
            s, u = steps(alpha, align, S)
            ws = np.max(rng.choice(s, (2000, 128)), axis=1).mean()
            wu = np.max(rng.choice(u, (2000, 128)), axis=1).mean()
            print(f"load {alpha:.3f} align {align} group {S}: per probe {s.mean():.3f} / {u.mean():.3f}, "
                  f"per wave of 128 {ws:.2f} / {wu:.2f} round trips (found / absent)")


if __name__ == "__main__":
    main()
