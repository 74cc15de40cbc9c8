"""Executable model of the parallel lazy engine, for tests only.

composeShortestPath (src/ops/compose-shortest-path.zig:26-401) for non-negative finite
weights, decomposed into order-independent pieces plus one ordering pass:

  1. the product lattice = compose.zig's (same 4 phases, same reachable tuples);
  2. dist = least fixpoint of d(X) = min fl(d(s) + w) (Dijkstra's values);
  3. lazy ids = first touch in (dist, id) pop order, computed in rounds: each round pops
     every open (touched, unpopped) node with the minimum dist, in id order -- any node
     touched meanwhile gets a larger id, so it pops after all of them -- and numbers the
     newly touched targets in (popper order, candidate order);
  4. back(X) = lexmin (source id, il, ol, candidate order) over tight in-arcs
     (relax at :107-141 is a lexicographic min on (dist, curr_id, il, ol); a full tie
     keeps the first relaxation, i.e. the earlier candidate of the same source);
  5. best = lexmin (total, id) over nodes whose two finals are non-Zero (:165-179);
  6. backtrace until the start id (:372-380; bounded: a cycle reports CYCLE).

`lazy_via_rounds` returns the same chain tuple as oracle_ffi.chain, plus the number of
rounds; the tests compare it with the oracle's own lazy replay.
"""
import math

import oracle_ffi as O


def lattice(lhs: O.Fst, blob: bytes):
    rc, lat = O.compose(lhs, blob)
    assert rc == O.OR_OK
    return lat


def fixpoint(lat: O.Fst):
    n = lat.num_states
    d = [math.inf] * n
    if lat.start == O.NO_STATE:
        return d
    d[lat.start] = 0.0
    changed = True
    while changed:
        changed = False
        for s in range(n):
            if d[s] == math.inf:
                continue
            for (_, _, w, x) in lat.arcs[s]:
                nd = d[s] + w if not (math.isinf(d[s]) or math.isinf(w)) else math.inf
                if nd < d[x]:
                    d[x] = nd
                    changed = True
    return d


def lazy_ids(lat: O.Fst, d):
    """First-touch ids in Dijkstra pop order, in parallel rounds.

    A node is poppable ("active") once a popped in-neighbour reaches it tightly (its
    tentative dist then equals its final d) -- the start from the outset.  With weights
    >= 0 the heap minimum is always an active node at the minimum active d (dmin).  A
    round pops the active nodes at dmin in id order, as a batch: popping u can activate
    an older node x (d(x) == dmin through a 0-weight arc) that must pop before any
    batch member with a larger id, so the batch is the longest id-ordered prefix that no
    earlier member's joiner undercuts.  Nodes first touched in the round get fresh ids,
    larger than all others: they never undercut."""
    n = lat.num_states
    lid = [None] * n
    lid[lat.start] = 0
    nxt = 1
    popped = [False] * n
    active = {lat.start}
    rounds = 0
    while active:
        rounds += 1
        dmin = min(d[u] for u in active)
        S = sorted((u for u in active if d[u] == dmin), key=lambda u: lid[u])
        # joiners of each member: older, inactive, unpopped targets it activates at dmin
        batch = []
        undercut = math.inf
        for u in S:
            if lid[u] > undercut:
                break
            batch.append(u)
            for (_, _, w, x) in lat.arcs[u]:
                if (lid[x] is not None and not popped[x] and x not in active and
                        d[u] + w == d[x] == dmin):
                    undercut = min(undercut, lid[x])
        for u in batch:
            popped[u] = True
            active.discard(u)
            for (_, _, w, x) in lat.arcs[u]:
                if lid[x] is None:
                    lid[x] = nxt
                    nxt += 1
                if not popped[x] and d[u] + w == d[x]:
                    active.add(x)
    return lid, rounds


def lazy_via_rounds(lhs: O.Fst, blob: bytes):
    lat = lattice(lhs, blob)
    if lat.start == O.NO_STATE:
        return None, 0
    d = fixpoint(lat)
    lid, rounds = lazy_ids(lat, d)
    n = lat.num_states
    back = [None] * n   # (lid(src), il, ol, cand, src, w)
    for s in range(n):
        if d[s] == math.inf:
            continue
        for ci, (il, ol, w, x) in enumerate(lat.arcs[s]):
            nd = d[s] + w
            if nd == d[x]:
                key = (lid[s], il, ol, ci, s, w)
                if back[x] is None or key[:4] < back[x][:4]:
                    back[x] = key
    best = None
    for x in range(n):
        fw = lat.finals[x]           # lattice final = fw1 (x) fw2, non-Zero iff both are
        if math.isinf(fw):
            continue
        total = d[x] + fw
        key = (total, lid[x])
        if best is None or key < best[0]:
            best = (key, x)
    if best is None:
        return None, rounds
    x = best[1]
    arcs = []
    for _ in range(n + 1):  # compose-shortest-path.zig:372-380: walk back to the start
        if x == lat.start:
            break
        if back[x] is None:
            return None, rounds
        _, il, ol, _, s, w = back[x]
        arcs.append((il, ol, w))
        x = s
    else:
        return "cycle", rounds
    arcs.reverse()
    return ([a[0] for a in arcs], [a[1] for a in arcs], [a[2] for a in arcs],
            lat.finals[best[1]]), rounds


# ---------------------------------------------------------------------------------
# Bucket replay (kernels/lazy_dense.hpp): the reference's own pop sequence, with the
# heap split into (a) the set of open tuples at the current distance dcur, as a bitmap
# over ids (pop = lowest set bit), and (b) an unsorted list of (dist, tuple) entries
# above dcur, scanned when the bitmap empties (dcur advances to the smallest valid
# entry; every valid entry at that distance moves into the bitmap).
# ---------------------------------------------------------------------------------
def lazy_via_buckets(labels, rhs: O.Fst, stats=None, early=False):
    """composeShortestPath(chain(labels), frozen(rhs), 1) for finite weights >= 0 and
    labels != 0.  Returns the oracle_ffi.chain tuple, None (empty) or "cycle".

    early: the band replay's exact early exit (kernels/lazy_band.hpp, DESIGN.md §4.2c;
    taken only when every final weight is >= 0 or Zero): stop before a pop at distance D
    once the best total is finite and either D > best total, or D == best total and every
    tuple with an id <= emax is settled, emax = the largest id on the best tuple's back
    chain (walked when the next pop passes the last emax)."""
    L = len(labels)
    NS = rhs.num_states
    if rhs.start == O.NO_STATE:
        return None
    # fromMutable sorts by (il, ol, w, next): arc.zig:46-54
    arcs = [sorted(a, key=lambda t: (t[0], t[1], t[2], t[3])) for a in rhs.arcs]
    idx_of = []                       # id -> (k, s, f)
    rec = {}                          # (k, s, f) -> [dist, id, settled, back]
    bucket = set()                    # ids open at dcur
    future = []                       # (dist, tuple)
    st = {"pops": 0, "advances": 0, "scanned": 0, "future_max": 0, "bucket_max": 0}

    def touch(t):
        r = rec.get(t)
        if r is None:
            r = [math.inf, len(idx_of), False, None]
            rec[t] = r
            idx_of.append(t)
            return r, True
        return r, False

    t0 = (0, rhs.start, 0)
    r0, _ = touch(t0)
    r0[0] = 0.0
    dcur = 0.0
    bucket.add(0)
    best = None                       # (total, id, fw)
    early = early and all(x >= 0 or math.isinf(x) for x in rhs.finals)
    emax = 0
    st["early_exit"] = False

    def chain_max(b_id):
        m, cur = b_id, b_id
        for _ in range(len(idx_of) + 1):
            if cur == 0:
                break
            back = rec[idx_of[cur]][3]
            cur = back[0]
            m = max(m, cur)
        return m

    while True:
        if not bucket:               # advance: scan + compact the future list
            st["advances"] += 1
            st["scanned"] += len(future)
            live = [(d, t) for (d, t) in future if not rec[t][2] and rec[t][0] == d]
            if not live:
                break
            dcur = min(d for d, _ in live)
            if early and best is not None and not math.isinf(best[0]) and dcur > best[0]:
                st["early_exit"] = True
                break
            future = [(d, t) for (d, t) in live if d != dcur]
            for d, t in live:
                if d == dcur:
                    bucket.add(rec[t][1])
        st["bucket_max"] = max(st["bucket_max"], len(bucket))
        pid = min(bucket)
        if (early and best is not None and not math.isinf(best[0]) and dcur == best[0]
                and pid > emax):
            live_ids = [rec[t][1] for (d, t) in future if not rec[t][2] and rec[t][0] == d]
            if not live_ids or min(live_ids) > emax:
                m = chain_max(best[1])
                if m <= emax:
                    st["early_exit"] = True
                    break
                emax = m
        bucket.discard(pid)
        st["pops"] += 1
        if stats is not None and "order" in stats:
            stats["order"].append(pid)
        t = idx_of[pid]
        r = rec[t]
        assert r[0] == dcur and not r[2]
        r[2] = True
        k, s, f = t
        fw1 = 0.0 if k == L else math.inf
        fw2 = rhs.finals[s]
        if not math.isinf(fw1) and not math.isinf(fw2):
            total = dcur + (fw1 + fw2)
            if best is None or total < best[0] or (total == best[0] and pid < best[1]):
                best = (total, pid, fw1 + fw2)
                emax = max(emax, pid)
        cands = []                    # (target, il, ol, w) in the reference's phase order
        if k < L:
            cands += [((k + 1, a[3], 0), a[0], a[1], 0.0 + a[2])
                      for a in arcs[s] if a[0] == labels[k]]
        if f != 2:
            cands += [((k, a[3], 0 if False else 1), 0, a[1], a[2])
                      for a in arcs[s] if a[0] == 0]
        for (x, il, ol, w) in cands:
            rx, new = touch(x)
            nd = dcur + w
            od = rx[0]
            take = math.isinf(od) or nd < od
            if not take and nd == od:
                b = rx[3]
                take = b is None or pid < b[0] or (pid == b[0] and (il, ol) < (b[1], b[2]))
            if not take:
                continue
            rx[0] = nd
            rx[3] = (pid, il, ol, w)
            if rx[2] or nd == od:
                continue                  # settled, or already queued at this distance
            if nd == dcur:
                bucket.add(rx[1])
            else:
                future.append((nd, x))
        st["future_max"] = max(st["future_max"], len(future))
    if stats is not None:
        stats.update(st)
    if best is None:
        return None
    out = []
    cur = best[1]
    for _ in range(len(idx_of) + 1):
        if cur == 0:
            break
        b = rec[idx_of[cur]][3]
        if b is None:
            return None
        out.append(b[1:])
        cur = b[0]
    else:
        return "cycle"
    out.reverse()
    return ([a[0] for a in out], [a[1] for a in out], [a[2] for a in out], best[2])
