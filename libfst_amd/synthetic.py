"""Synthetic stand-ins for config 4 (WeTextProcessing tagger -> verbalizer).

The real zh_tagger.fst / zh_verbalizer.fst are not available offline, so
bench and tests use two small byte-level transducers with the same shape of work: label =
byte + 1 (compileString, src/string.zig:24-50), epsilon-input arcs for multi-symbol
outputs (rhs epsilons), and an ambiguous choice resolved by weight.

  tagger      copies letters and spaces; a digit d is either copied (weight 1.0) or
              tagged as "#" + chr(ord('a') + d) (weight 0.5, via an epsilon-input arc);
  verbalizer  copies letters, spaces and digits; "#x" becomes the English word of digit
              x, written with an epsilon-input chain.

Builders return plain lists (num_states, start, finals, arcs per state as (il, ol, w,
next)); tests wrap them for the oracle, bench freezes them through the C ABI.
"""
INF = float("inf")
LETTERS = "abcdefghijklmnopqrstuvwxyz "
DIGITS = "0123456789"
WORDS = ["zero", "one", "two", "three", "four", "five", "six", "seven", "eight", "nine"]


def lab(ch: str) -> int:
    return ord(ch) + 1


class _Builder:
    def __init__(self):
        self.finals = []
        self.arcs = []

    def state(self, final=INF):
        self.finals.append(final)
        self.arcs.append([])
        return len(self.finals) - 1

    def arc(self, s, il, ol, w, nx):
        self.arcs[s].append((il, ol, float(w), nx))

    def lists(self):
        return len(self.finals), 0, list(self.finals), [list(a) for a in self.arcs]


def tagger():
    b = _Builder()
    s0 = b.state(0.0)
    for ch in LETTERS:
        b.arc(s0, lab(ch), lab(ch), 0.0, s0)
    for d, ch in enumerate(DIGITS):
        b.arc(s0, lab(ch), lab(ch), 1.0, s0)          # keep the digit
        mid = b.state()
        b.arc(s0, lab(ch), lab("#"), 0.5, mid)        # tag it ...
        b.arc(mid, 0, lab(chr(ord("a") + d)), 0.0, s0)  # ... as "#" + letter
    return b.lists()


def verbalizer():
    b = _Builder()
    s0 = b.state(0.0)
    for ch in LETTERS + DIGITS:
        b.arc(s0, lab(ch), lab(ch), 0.0, s0)
    hs = b.state()
    b.arc(s0, lab("#"), 0, 0.0, hs)
    for d, word in enumerate(WORDS):
        cur = b.state()
        b.arc(hs, lab(chr(ord("a") + d)), 0, 0.0, cur)
        for k, ch in enumerate(word):
            nxt = s0 if k == len(word) - 1 else b.state()
            b.arc(cur, 0, lab(ch), 0.0, nxt)
            cur = nxt
    return b.lists()


def utterances(rng, n, min_len=5, max_len=40):
    """Random texts of letters, spaces and digit runs (numpy Generator `rng`)."""
    alphabet = LETTERS + DIGITS * 2
    out = []
    for _ in range(n):
        L = int(rng.integers(min_len, max_len + 1))
        out.append("".join(alphabet[int(i)] for i in rng.integers(0, len(alphabet), L)))
    return out


def to_labels(texts):
    """CSR (labels u32, offsets u64) of compileString label sequences."""
    import numpy as np
    lens = [len(t) for t in texts]
    offsets = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    labels = np.fromiter((ord(c) + 1 for t in texts for c in t), dtype=np.uint32,
                         count=int(offsets[-1]))
    return labels, offsets


def to_mutable(spec):
    """A libfst_amd.MutableFst from builder lists (C ABI)."""
    from .fst import MutableFst
    ns, start, finals, arcs = spec
    m = MutableFst()
    for _ in range(ns):
        m.add_state()
    m.set_start(start)
    for s, fw in enumerate(finals):
        if fw != INF:
            m.set_final(s, fw)
    for s, al in enumerate(arcs):
        for (il, ol, w, nx) in al:
            m.add_arc(s, il, ol, w, nx)
    return m
