"""Executable model of a layer-local lazy engine (composeShortestPath on layered lattices).

For tests only.  Domain: chain inputs without label 0 against an rhs without input
epsilons, finite weights >= 0 -- every lattice arc goes from layer k to layer k+1.
The reference (src/ops/compose-shortest-path.zig:26-401) pops min (dist, id), ids given
at first touch (getOrCreate, :70-89).  Claim modelled here:

  C  If every tuple x (but the start) has a tight in-neighbour u that pops before it --
     d(u) < d(x), or d(u) == d(x) and id(u) < id(x) -- then the pop order is exactly the
     sort by (dist, id) (the heap minimum is then always the next tuple of that order).

Under C everything the answer needs is layer-local:
  * p_k  = pop rank within layer k = rank of (d, r_k);
  * r_k+1 (id order within layer k+1) = order of (p_k(u*), j*) where u* is x's first
    toucher -- the in-neighbour popped first -- and j* its candidate position;
  * back(x) = lexmin (r_k(u), ol, j) over tight in-arcs (relax :107-141);
  * best = lexmin (total, r_L) (:165-179).
C itself needs id(u) < id(x) across adjacent layers.  id(u) < id(x) iff u's first toucher
popped before x's, recursively down the chains of first touchers; the chain of distances
(d(u*), d(u**), ...) is non-increasing, so each tuple keeps tb = d(u*) and run = the
length of the initial run of equal values in its chain: with tb equal, the shorter run
means the chain drops (or reaches the start) first, i.e. the earlier touch.  Equal tb and
equal run is undecided: the model reports FALLBACK (the GPU engine hands such a string to
the rounds engine).
"""
import math
import struct

import numpy as np

FALLBACK = "fallback"


def parse_blob(blob: bytes):
    magic, ver, wt, fl, ns, na, start, _ = struct.unpack_from("<IHBBIIII", blob, 0)
    st = np.frombuffer(blob, dtype=np.dtype([("off", "<u4"), ("n", "<u4"), ("fin", "<f8")]),
                       count=ns, offset=24)
    arcs = np.frombuffer(blob, dtype=np.dtype([("il", "<u4"), ("ol", "<u4"), ("w", "<f8"),
                                               ("nx", "<u4"), ("pad", "<u4")]),
                         count=na, offset=24 + 16 * ns)
    return ns, start, st, arcs


def arcs_by_ilabel(st, arcs, s, lab):
    o, n = int(st[s]["off"]), int(st[s]["n"])
    return [(j, int(arcs[a]["ol"]), float(arcs[a]["w"]), int(arcs[a]["nx"]))
            for j, a in enumerate(x for x in range(o, o + n) if int(arcs[x]["il"]) == lab)]


def times(a, b):
    return math.inf if (math.isinf(a) or math.isinf(b)) else a + b


def lazy_pull(blob: bytes, labels):
    """-> (status, ilabels, olabels, weights, final); status 'ok' | 'empty' | FALLBACK."""
    ns, start, st, arcs = parse_blob(blob)
    if start == 0xFFFFFFFF:
        return ("empty", [], [], [], None)
    # layer cells: state -> dict(d, r, p, tb, run, back=(state, j, ol, w))
    layer = {start: dict(d=0.0, r=0, p=0, tb=None, run=0, back=None)}
    layers = [layer]
    for k, lab in enumerate(labels):
        inarcs = {}
        for u, cu in layer.items():
            for (j, ol, w, nx) in arcs_by_ilabel(st, arcs, u, lab):
                inarcs.setdefault(nx, []).append((u, j, ol, w))
        nxt = {}
        for t, lst in inarcs.items():
            d = min(times(layer[u]["d"], w) for (u, j, ol, w) in lst)
            us, js, _, _ = min(lst, key=lambda a: (layer[a[0]]["p"], a[1]))
            back = min((a for a in lst if times(layer[a[0]]["d"], a[3]) == d),
                       key=lambda a: (layer[a[0]]["r"], a[2], a[1]))
            cu = layer[us]
            tb = cu["d"]
            run = 1 + (cu["run"] if cu["tb"] is not None and cu["tb"] == tb else 0)
            nxt[t] = dict(d=d, key=(cu["p"], js), tb=tb, run=run, back=back)
        if not nxt:
            return ("empty", [], [], [], None)
        for rank, t in enumerate(sorted(nxt, key=lambda t: nxt[t]["key"])):
            nxt[t]["r"] = rank
        for rank, t in enumerate(sorted(nxt, key=lambda t: (nxt[t]["d"], nxt[t]["r"]))):
            nxt[t]["p"] = rank
        # condition C for every tuple of the new layer
        for t, c in nxt.items():
            ok = False
            for (u, j, ol, w) in inarcs[t]:
                cu = layer[u]
                if times(cu["d"], w) != c["d"]:
                    continue  # not tight
                if u == start and k == 0:
                    ok = True  # id 0
                elif cu["d"] < c["d"]:
                    ok = True
                elif cu["tb"] < c["tb"] or (cu["tb"] == c["tb"] and cu["run"] < c["run"]):
                    ok = True
                if ok:
                    break
            if not ok:
                return (FALLBACK, [], [], [], None)
        layer = nxt
        layers.append(layer)
    # best final (layer L, lhs final One): lexmin (d + fw2, r)
    best = None
    for t, c in layer.items():
        fw = float(st[t]["fin"])
        if math.isinf(c["d"]) or math.isinf(fw):
            continue
        key = (times(c["d"], fw), c["r"])
        if best is None or key < best[0]:
            best = (key, t, fw)
    if best is None:
        return ("empty", [], [], [], None)
    il, ol, ws = [], [], []
    t = best[1]
    for k in range(len(labels), 0, -1):
        u, j, o, w = layers[k][t]["back"]
        il.append(labels[k - 1])
        ol.append(o)
        ws.append(w)
        t = u
    return ("ok", il[::-1], ol[::-1], ws[::-1], best[2])
