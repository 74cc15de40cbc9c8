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
