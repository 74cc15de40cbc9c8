"""WeText-scale synthetic stand-in for config 4 (zh tagger -> verbalizer), generated.

The real WeTextProcessing zh_tagger.fst / zh_verbalizer.fst are unavailable offline
(SURVEY.md §8c), and the toy stand-ins of libfst_amd.synthetic are 21 / 45 states.  This
module generates a tagger with the structure that matters to the engines at WeText scale
(deterministic for a seed; sizes at the defaults in brackets):

  * UTF-8 byte labels (label = byte + 1, as att2lfst leaves a byte-tokenized asset and
    fst_compile_string encodes the input, src/string.zig:24-50; src/tools/att2lfst.zig);
  * a pass-through path for ~3,500 CJK characters (a byte trie: lead byte -> 64-way
    middle-byte states -> last byte back to the root) and printable ASCII, 1.0 per char;
  * a lexicon of ~32,000 words of 2-4 CJK characters: an input trie that deletes the word
    (ilabel byte, olabel epsilon; 0.4 per char, so a lexicon word beats pass-through), and
    at each word end an epsilon-input output chain writing "w{" + replacement + "}" (the
    replacement: 1-3 CJK characters): rhs input epsilons, long epsilon-output chains;
  * "determinized union" fallback arcs: at every character boundary inside the lexicon
    trie, arcs on every lead byte and every ASCII digit leave the word (penalty 2.0) --
    multi-label states of dozens of arcs;
  * a number class: ASCII digit runs become "n{" + digits + "}" (epsilon-input chains);
  * state ids scattered by a random permutation: no banded structure, P / LP windows of
    the metric shape do not apply.

[~0.43 M states, ~1.03 M arcs]  The verbalizer undoes the markup: "w{...}" and "n{...}"
are deleted around their content, digits inside "n{...}" become Chinese numerals (3-byte
epsilon-input chains), everything else passes through (a few thousand states).

Builders return numpy arrays; `freeze_blob` packs them exactly as Fst.fromMutable
(src/fst.zig:160-224: per-state stable sort by compareByIlabel, src/arc.zig:46-54), so the
blob is byte-identical to fst_freeze of the same MutableFst (tests check it against the
oracle's freeze).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

INF = float("inf")
NUMERALS = "零一二三四五六七八九"


@dataclass
class Graph:
    num_states: int
    start: int
    finals: np.ndarray   # f64 [ns], inf = not final
    src: np.ndarray      # u32 [na]  arcs in insertion order
    il: np.ndarray
    ol: np.ndarray
    w: np.ndarray        # f64
    dst: np.ndarray

    def lists(self):
        """(num_states, start, finals, arcs per state) like libfst_amd.synthetic builders."""
        arcs = [[] for _ in range(self.num_states)]
        for s, a, b, w, d in zip(self.src.tolist(), self.il.tolist(), self.ol.tolist(),
                                 self.w.tolist(), self.dst.tolist()):
            arcs[s].append((a, b, w, d))
        return self.num_states, self.start, self.finals.tolist(), arcs


class _B:
    """Arc list builder with growable numpy-friendly python lists."""

    def __init__(self):
        self.nstates = 0
        self.finals = []
        self.src, self.il, self.ol, self.w, self.dst = [], [], [], [], []

    def state(self, final=INF):
        self.finals.append(final)
        self.nstates += 1
        return self.nstates - 1

    def arc(self, s, il, ol, w, d):
        self.src.append(s)
        self.il.append(il)
        self.ol.append(ol)
        self.w.append(w)
        self.dst.append(d)

    def chain_out(self, s, data: bytes, d, w=0.0):
        """epsilon-input chain from s writing `data`, ending in d."""
        cur = s
        for i, byte in enumerate(data):
            nxt = d if i == len(data) - 1 else self.state()
            self.arc(cur, 0, byte + 1, w if i == 0 else 0.0, nxt)
            cur = nxt

    def graph(self, start, permute_seed=None) -> Graph:
        g = Graph(self.nstates, start, np.asarray(self.finals, np.float64),
                  np.asarray(self.src, np.uint32), np.asarray(self.il, np.uint32),
                  np.asarray(self.ol, np.uint32), np.asarray(self.w, np.float64),
                  np.asarray(self.dst, np.uint32))
        if permute_seed is not None:  # scatter the state ids
            perm = np.random.default_rng(permute_seed).permutation(g.num_states).astype(np.uint32)
            fin = np.empty_like(g.finals)
            fin[perm] = g.finals
            g = Graph(g.num_states, int(perm[start]), fin, perm[g.src], g.il, g.ol, g.w,
                      perm[g.dst])
        return g


def cjk_chars(rng, n):
    """n distinct CJK unified ideographs (U+4E00..U+9FA5), the numerals first."""
    base = [ord(c) for c in NUMERALS + "十百千万亿"]
    pool = np.setdiff1d(np.arange(0x4E00, 0x9FA6), np.asarray(base))
    pick = rng.choice(pool, size=n - len(base), replace=False)
    return [chr(c) for c in base] + [chr(int(c)) for c in pick]


ASCII = [chr(c) for c in range(0x20, 0x7F)]


def _pass_through(b: _B, root, chars, w_char=1.0):
    """byte trie from root over `chars`' UTF-8 encodings, each char costs w_char, copies."""
    first = {}   # lead byte -> state
    mid = {}     # (lead, mid byte) -> state
    for ch in chars:
        u = ch.encode("utf-8")
        if len(u) == 1:
            b.arc(root, u[0] + 1, u[0] + 1, w_char, root)
            continue
        assert len(u) == 3
        if u[0] not in first:
            first[u[0]] = b.state()
            b.arc(root, u[0] + 1, u[0] + 1, w_char, first[u[0]])
        if (u[0], u[1]) not in mid:
            mid[(u[0], u[1])] = b.state()
            b.arc(first[u[0]], u[1] + 1, u[1] + 1, 0.0, mid[(u[0], u[1])])
        b.arc(mid[(u[0], u[1])], u[2] + 1, u[2] + 1, 0.0, root)
    return first


def tagger(seed=2024, n_chars=3500, n_words=32000) -> Graph:
    rng = np.random.default_rng(seed)
    chars = cjk_chars(rng, n_chars)
    b = _B()
    root = b.state(0.0)
    first = _pass_through(b, root, chars + ASCII)
    leads = sorted(first)
    digits = [ord(c) for c in "0123456789"]
    # number class: root -digit-> chain "n{" then digits, "}" on leaving
    nopen = b.state()
    b.chain_out(root, b"n{", nopen, 0.0)
    nrun = b.state()
    for d in digits:
        b.arc(nopen, d + 1, d + 1, 0.3, nrun)
        b.arc(nrun, d + 1, d + 1, 0.3, nrun)
    b.chain_out(nrun, b"}", root, 0.0)
    # lexicon: input trie (deletes), fallback arcs at char boundaries, output chains
    trie = {}
    for _ in range(n_words):
        k = int(rng.integers(2, 5))
        word = "".join(chars[int(i)] for i in rng.integers(10, n_chars, k))
        repl = "".join(chars[int(i)] for i in rng.integers(10, n_chars, int(rng.integers(1, 4))))
        cur = root
        u = word.encode("utf-8")
        for i, byte in enumerate(u):
            key = (cur, byte)
            if key not in trie:
                nxt = b.state()
                trie[key] = nxt
                b.arc(cur, byte + 1, 0, 0.4 if i % 3 == 0 else 0.0, nxt)
                if i % 3 == 2 and i + 1 < len(u):  # a char boundary inside the word
                    for ld in leads:
                        b.arc(nxt, ld + 1, ld + 1, 2.0, first[ld])
                    for d in digits:
                        b.arc(nxt, d + 1, d + 1, 2.0, root)
            cur = trie[key]
        b.chain_out(cur, b"w{" + repl.encode("utf-8") + b"}", root, 0.0)
    return b.graph(root, permute_seed=seed + 1)


def verbalizer(seed=2024, n_chars=3500) -> Graph:
    rng = np.random.default_rng(seed)
    chars = cjk_chars(rng, n_chars)
    b = _B()
    root = b.state(0.0)
    _pass_through(b, root, chars + [c for c in ASCII if c not in "nw{}"], w_char=0.0)
    for c in "nw":  # letters n / w not followed by "{" copy through
        s = b.state()
        b.arc(root, ord(c) + 1, 0, 0.0, s)
        b.chain_out(s, c.encode(), root, 0.5)
    # "w{" ... "}": markup deleted, content (CJK pass-through) copied
    wopen = b.state()
    b.arc(root, ord("w") + 1, 0, 0.0, wopen)
    win = b.state()
    b.arc(wopen, ord("{") + 1, 0, 0.0, win)
    _pass_through(b, win, chars, w_char=0.0)  # content returns to `win`
    b.arc(win, ord("}") + 1, 0, 0.0, root)
    # "n{" digits "}": digits -> numerals
    nopen = b.state()
    b.arc(root, ord("n") + 1, 0, 0.0, nopen)
    nin = b.state()
    b.arc(nopen, ord("{") + 1, 0, 0.0, nin)
    for d in range(10):
        mid = b.state()
        b.arc(nin, ord(str(d)) + 1, 0, 0.0, mid)
        b.chain_out(mid, NUMERALS[d].encode("utf-8"), nin, 0.0)
    b.arc(nin, ord("}") + 1, 0, 0.0, root)
    return b.graph(root, permute_seed=seed + 2)


def utterances(rng, n, tag: Graph | None = None, seed=2024, n_chars=3500, n_words=32000,
               min_chars=4, max_chars=24):
    """Mixed utterances: CJK characters, lexicon words (re-generated from the seed), digit
    runs and ASCII words; returned as CSR (labels u32 = byte + 1, offsets u64)."""
    g = np.random.default_rng(seed)
    chars = cjk_chars(g, n_chars)
    words = []
    for _ in range(min(n_words, 2000)):  # the tagger's first words (same draws)
        k = int(g.integers(2, 5))
        words.append("".join(chars[int(i)] for i in g.integers(10, n_chars, k)))
        g.integers(10, n_chars, int(g.integers(1, 4)))
    out = []
    for _ in range(n):
        parts, total = [], 0
        goal = int(rng.integers(min_chars, max_chars + 1))
        while total < goal:
            r = rng.random()
            if r < 0.55:
                t = chars[int(rng.integers(0, n_chars))]
            elif r < 0.8:
                t = words[int(rng.integers(0, len(words)))]
            elif r < 0.92:
                t = "".join(str(int(x)) for x in rng.integers(0, 10, int(rng.integers(1, 6))))
            else:
                t = "".join(chr(int(x)) for x in rng.integers(0x61, 0x7B, int(rng.integers(1, 5))))
            parts.append(t)
            total += len(t)
        out.append("".join(parts).encode("utf-8"))
    lens = np.fromiter((len(u) for u in out), np.int64, len(out))
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    labels = np.frombuffer(b"".join(out), np.uint8).astype(np.uint32) + 1
    return labels, offsets


def freeze_blob(g: Graph, weight_type: int = 0) -> bytes:
    """Fst.fromMutable (src/fst.zig:160-224) of the graph, as blob bytes."""
    ns, na = g.num_states, len(g.src)
    # stable per-state sort by (ilabel, olabel, weight, nextstate) = compareByIlabel
    order = np.lexsort((g.dst, g.w, g.ol, g.il, g.src))
    counts = np.bincount(g.src, minlength=ns).astype(np.uint32)
    offs = np.zeros(ns, np.uint32)
    offs[1:] = np.cumsum(counts)[:-1]
    header = np.zeros(1, dtype=[("magic", "<u4"), ("version", "<u2"), ("wt", "u1"), ("flags", "u1"),
                                ("ns", "<u4"), ("na", "<u4"), ("start", "<u4"), ("pad", "<u4")])
    header[0] = (0x46535421, 1, weight_type, 0, ns, na, g.start, 0)
    st = np.zeros(ns, dtype=[("off", "<u4"), ("n", "<u4"), ("final", "<f8")])
    st["off"], st["n"], st["final"] = offs, counts, g.finals
    arcs = np.zeros(na, dtype=[("il", "<u4"), ("ol", "<u4"), ("w", "<f8"), ("next", "<u4"),
                               ("pad", "<u4")])
    arcs["il"], arcs["ol"], arcs["w"], arcs["next"] = (g.il[order], g.ol[order], g.w[order],
                                                       g.dst[order])
    return header.tobytes() + st.tobytes() + arcs.tobytes()
