"""Simulation of SearchByProjection's sequential claim replay (H5) and of two parallel
forms, on random candidate lists: the chunked Jacobi fixpoint of k_seq_commit /
proj_replay (64 queries per chunk; round 3 with non-blocking acceptances as sequence
points, round 4 without, its claims written as the kernel writes them) and a
sliding-window form (lanes retire as soon as every earlier lane is certified, and take
the next query).  Checks both against the
sequential loop and counts iterations.  TEST / DESIGN TOOLING ONLY.

    python tools/sim/replay_sim.py [--scenes 300] [--seed 0]
"""
from __future__ import annotations

import argparse
import random

K = 12          # listed entries per query (kTopK)
TH = 50         # acceptance threshold (TH_HIGH-like)
NONE, TRUNC = ("none",), ("trunc",)


def make_scene(rng, nq, npos, ratio, blocked_frac, dens):
    """Per query its full candidate set [(dist, pos, oct)] sorted by (dist, pos)."""
    qs = []
    for _ in range(nq):
        c = rng.randrange(npos)
        m = max(1, int(rng.expovariate(1.0 / dens)))
        cands = {}
        for _ in range(m):
            p = min(npos - 1, max(0, c + rng.randrange(-8, 9)))
            cands[p] = (rng.randrange(0, 90), p, rng.randrange(0, 3))
        qs.append(sorted(cands.values()))
    bself = [rng.random() >= blocked_frac for _ in range(nq)]  # claim blocks later queries
    return qs, bself


def choose(lst, blocked, ratio, nnratio=0.9):
    """(accepted entry or None) given the full candidate list and the blocked positions:
    the reference's loop (best / second best over unblocked candidates)."""
    free = [e for e in lst if e[1] not in blocked]
    if not free:
        return None
    a1 = free[0]
    if a1[0] > TH:
        return None
    if ratio:
        a2 = free[1] if len(free) > 1 else None
        lvl2 = a2[2] if a2 else -1
        d2 = a2[0] if a2 else 256
        if a1[2] == lvl2 and a1[0] > nnratio * d2:
            return None
    return a1


def sequential(qs, bself, ratio):
    blocked, out = set(), []
    for q, lst in enumerate(qs):
        a = choose(lst, blocked, ratio)
        out.append(a)
        if a is not None and bself[q]:
            blocked.add(a[1])
    return out


def final_claims(qs, out):
    """The keypoint -> query map the reference leaves in F.mvpMapPoints: every acceptance
    writes its keypoint, so the last one in query order keeps it (ORBmatcher.cc:167)."""
    m = {}
    for q, a in enumerate(out):
        if a is not None:
            m[a[1]] = q
    return m


class Lane:
    """A query's listed entries (the first K of its candidates against the claims of some
    moment) and its current choice."""

    def __init__(self, q, qs, blocked):
        self.q = q
        self.relist(qs, blocked)

    def relist(self, qs, blocked):
        free = [e for e in qs[self.q] if e[1] not in blocked]
        self.e = free[:K]
        self.full = len(free) > K
        self.sig = None


def evaluate(lane, blocked_pos, ratio):
    """The kernel's eval: c1 / acceptance / exhausted against the blocked positions."""
    need = 2 if ratio else 1
    fm = [e for e in lane.e if e[1] not in blocked_pos]
    x = lane.full and len(fm) < need
    lastgt = lane.e and lane.e[-1][0] > TH
    if x and ((len(fm) == 0 and lastgt) or (len(fm) == 1 and fm[0][0] > TH)):
        x = False
    if x:
        return TRUNC
    if not fm or fm[0][0] > TH:
        return NONE
    a1 = fm[0]
    if ratio:
        a2 = fm[1] if len(fm) > 1 else None
        lvl2 = a2[2] if a2 else -1
        d2 = a2[0] if a2 else 256
        if a1[2] == lvl2 and a1[0] > 0.9 * d2:
            return NONE
    return a1


def sliding(qs, bself, ratio, W=64):
    """Sliding window: lanes hold queries F..F+W-1; each iteration every lane re-evaluates
    against the committed claims + the proposals of earlier lanes (previous iteration);
    the lanes before the first one whose choice changed are certified; they commit up to
    the first sequence point (exhausted list: re-scored against the claims; non-blocking
    acceptance: commits, then the lanes after it re-evaluate) and the window slides."""
    nq = len(qs)
    committed = set()
    out = [None] * nq
    lanes = {}
    F, nxt, iters = 0, 0, 0
    prop = {}  # q -> proposed position (previous iteration)
    while F < nq:
        while nxt < nq and nxt < F + W:
            lanes[nxt] = Lane(nxt, qs, committed)
            nxt += 1
        iters += 1
        # owner map from the previous iteration's proposals: position -> lowest q
        owner = {}
        for q, p in prop.items():
            if p is not None and (p not in owner or q < owner[p]):
                owner[p] = q
        newprop, first_change = {}, None
        for q in range(F, nxt):
            L = lanes[q]
            blocked = committed | {p for p, o in owner.items() if o < q}
            s = evaluate(L, blocked, ratio)
            if s != L.sig and first_change is None:
                first_change = q
            L.sig = s
            newprop[q] = s[1] if (s not in (NONE, TRUNC) and bself[q]) else None
        prop = newprop
        c = first_change if first_change is not None else nxt
        # commit the certified prefix [F, c) up to the first sequence point
        q = F
        while q < c:
            L = lanes[q]
            if L.sig is TRUNC:  # re-score against the committed claims, continue next iteration
                L.relist(qs, committed)
                prop.pop(q, None)
                break
            if L.sig not in (NONE, TRUNC):
                out[q] = L.sig
                if bself[q]:
                    committed.add(L.sig[1])
            prop.pop(q, None)
            del lanes[q]
            q += 1
            F = q
            if out[q - 1] is not None and not bself[q - 1]:
                # a non-blocking acceptance: fine, later lanes never saw it as a proposal
                pass
    return out, iters


def chunked(qs, bself, ratio, W=64):
    """The shipped form: chunks of W; iterate to a full fixpoint, commit, handle the
    sequence point, resume (iterations counted like the kernel's)."""
    nq = len(qs)
    committed = set()
    out = [None] * nq
    iters = 0
    for base in range(0, nq, W):
        qrange = list(range(base, min(nq, base + W)))
        lanes = {q: Lane(q, qs, committed) for q in qrange}
        start = base
        while start < qrange[-1] + 1:
            changed = True
            prop = {}
            while changed:
                iters += 1
                owner = {}
                for q, p in prop.items():
                    if p is not None and (p not in owner or q < owner[p]):
                        owner[p] = q
                changed, newprop = False, {}
                for q in range(start, qrange[-1] + 1):
                    L = lanes[q]
                    blocked = committed | {p for p, o in owner.items() if o < q}
                    s = evaluate(L, blocked, ratio)
                    if s != L.sig:
                        changed = True
                    L.sig = s
                    newprop[q] = s[1] if (s not in (NONE, TRUNC) and bself[q]) else None
                prop = newprop
            q = start
            while q <= qrange[-1]:
                L = lanes[q]
                if L.sig is TRUNC:
                    L.relist(qs, committed)
                    L.sig = None
                    break
                if L.sig is not NONE:
                    out[q] = L.sig
                    if bself[q]:
                        committed.add(L.sig[1])
                q += 1
                if out[q - 1] is not None and not bself[q - 1]:
                    break
            start = q
    return out, iters


def chunked_nb(qs, bself, ratio, W=64):
    """The round-4 form: like chunked, but a non-blocking acceptance does not stop the
    commit; the claims are written as the kernel writes them -- blocking ones directly,
    a non-blocking one only when no later lane of the same commit claims its keypoint.
    Returns (acceptances, final keypoint -> query map, iterations)."""
    nq = len(qs)
    committed = set()
    out = [None] * nq
    claims = {}
    iters = 0
    for base in range(0, nq, W):
        qrange = list(range(base, min(nq, base + W)))
        lanes = {q: Lane(q, qs, committed) for q in qrange}
        start = base
        while start < qrange[-1] + 1:
            changed = True
            prop = {}
            while changed:
                iters += 1
                owner = {}
                for q, p in prop.items():
                    if p is not None and (p not in owner or q < owner[p]):
                        owner[p] = q
                changed, newprop = False, {}
                for q in range(start, qrange[-1] + 1):
                    L = lanes[q]
                    blocked = committed | {p for p, o in owner.items() if o < q}
                    s = evaluate(L, blocked, ratio)
                    if s != L.sig:
                        changed = True
                    L.sig = s
                    newprop[q] = s[1] if (s not in (NONE, TRUNC) and bself[q]) else None
                prop = newprop
            f = next((q for q in range(start, qrange[-1] + 1) if lanes[q].sig is TRUNC), qrange[-1] + 1)
            com = [q for q in range(start, f) if lanes[q].sig is not NONE]
            last = {}
            for q in com:  # the dedup pass: the highest committing lane per keypoint
                last[lanes[q].sig[1]] = q
            for q in com:
                out[q] = lanes[q].sig
                p = lanes[q].sig[1]
                if bself[q]:
                    committed.add(p)
                    claims[p] = q
                elif last[p] == q:
                    claims[p] = q
            if f <= qrange[-1]:
                lanes[f].relist(qs, committed)
                lanes[f].sig = None
            start = f
    return out, claims, iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=300)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    rng = random.Random(a.seed)
    tot_s = tot_c = tot_n = 0
    for i in range(a.scenes):
        nq = rng.choice([64, 200, 1000])
        ratio = rng.random() < 0.5
        qs, bself = make_scene(rng, nq, nq * rng.choice([1, 2, 4]), ratio, rng.choice([0.0, 0.1, 0.5]),
                               rng.choice([4, 12, 30]))
        ref = sequential(qs, bself, ratio)
        s, it_s = sliding(qs, bself, ratio)
        c, it_c = chunked(qs, bself, ratio)
        n, cl, it_n = chunked_nb(qs, bself, ratio)
        assert s == ref, ("sliding", i)
        assert c == ref, ("chunked", i)
        assert n == ref and cl == final_claims(qs, ref), ("chunked_nb", i)
        tot_s += it_s
        tot_c += it_c
        tot_n += it_n
    print(f"{a.scenes} scenes: all equal to the sequential loop; iterations chunked (round 3) {tot_c}, "
          f"chunked with non-blocking commits (round 4) {tot_n}, sliding {tot_s}")


if __name__ == "__main__":
    main()


def profile(nq=1000, dens=12, blocked_frac=0.0, ratio=False, npos_mul=1, seeds=5):
    """Mean iterations of both forms on one scene family."""
    rs, rc = [], []
    for sd in range(seeds):
        rng = random.Random(1000 + sd)
        qs, bself = make_scene(rng, nq, nq * npos_mul, ratio, blocked_frac, dens)
        ref = sequential(qs, bself, ratio)
        s, it_s = sliding(qs, bself, ratio)
        c, it_c = chunked(qs, bself, ratio)
        assert s == ref and c == ref
        rs.append(it_s)
        rc.append(it_c)
    return sum(rc) / seeds, sum(rs) / seeds
