"""Blob ingestion: AT&T text -> frozen blob, binary load/save.  CPU only.

* fst_read_text (src/io/text.zig:20-115) against the oracle's restatement (read_att);
* tools/att2lfst and fst_load_att (src/tools/att2lfst.zig:54-60: +1 on every non-epsilon
  label, then fromMutable) byte-identical to the oracle's freeze of the shifted graph, on
  the reference's own corpus (tests/golden/corpus, byte copies of tests/corpus/*.att);
* fst_load reads the file into the blob's own (pinned when a GPU is present) block:
  load -> save round trips byte-identically, bad files are rejected like Fst.fromBytes.
"""
import os
import subprocess
import tempfile

import numpy as np
import pytest

import libfst_amd as F
import oracle_ffi as O

CORPUS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "corpus")
TOOL = os.path.join(os.path.dirname(F.fst.LIB_PATH), "att2lfst")
ATT_FILES = sorted(f for f in os.listdir(CORPUS) if f.endswith(".att"))


def shifted(f: O.Fst) -> O.Fst:
    g = O.Fst(start=f.start, finals=list(f.finals))
    g.arcs = [[(il + 1 if il else 0, ol + 1 if ol else 0, w, d) for (il, ol, w, d) in al]
              for al in f.arcs]
    return g


def lists(m: F.MutableFst):
    return m.to_lists()


def write(tmp, name, text):
    p = os.path.join(tmp, name)
    with open(p, "w") as fh:
        fh.write(text)
    return p


@pytest.mark.parametrize("name", ATT_FILES)
def test_read_text_matches_oracle(name):
    path = os.path.join(CORPUS, name)
    ref = O.read_att(open(path).read())
    start, finals, arcs = F.MutableFst.read_text(path).to_lists()
    assert start == ref.start
    assert finals == ref.finals
    assert arcs == ref.arcs


@pytest.mark.parametrize("name", ATT_FILES)
def test_att2lfst_tool_byte_identical(name, tmp_path):
    src = os.path.join(CORPUS, name)
    out = str(tmp_path / "out.fst")
    r = subprocess.run([TOOL, "--input", src, "--output", out], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "Converted" in r.stderr
    expect = O.freeze(shifted(O.read_att(open(src).read())))
    assert open(out, "rb").read() == expect
    # fst_load_att is the same conversion without the file round trip
    h = F.Fst.load_att(src)
    p2 = str(tmp_path / "out2.fst")
    h.save(p2)
    assert open(p2, "rb").read() == expect
    # and the unshifted variant is the plain freeze
    p3 = str(tmp_path / "out3.fst")
    F.Fst.load_att(src, shift_byte_labels=False).save(p3)
    assert open(p3, "rb").read() == O.freeze(O.read_att(open(src).read()))


def test_att_forms_and_errors(tmp_path):
    text = ("0 1 97 98 0.5\n"      # full arc
            "1\t2\t3\n"             # olabel = ilabel, weight One
            "2 3 4 2.25\n"          # fourth field is a weight (olabel = ilabel)
            "\r\n  \n"              # blank lines, CRLF
            "3 4\n"                 # "src dest": an integer second field is a final weight
            "4 Infinity\n"          # final Zero
            "5 inf\n"
            "4 0 0 0 0\r\n"         # epsilon arc back to the start
            "6\n")                  # final One
    p = write(str(tmp_path), "forms.att", text)
    ref = O.read_att(text)
    assert F.MutableFst.read_text(p).to_lists() == (ref.start, ref.finals, ref.arcs)
    for bad in ("x 1 2 3\n", "0 1 a 2\n", "0 1 2 3 4 5\n", "0 1.5 7\n", "0 -1 2 3\n",
                "4294967296 1 2\n", "4294967295 1 2\n", "0 4294967295 7\n"):
        pb = write(str(tmp_path), "bad.att", bad)
        with pytest.raises(ValueError):
            F.MutableFst.read_text(pb)
        with pytest.raises(ValueError):
            F.Fst.load_att(pb)
    r = subprocess.run([TOOL, "--input", pb, "--output", str(tmp_path / "x.fst")],
                       capture_output=True, text=True)
    assert r.returncode == 1
    r = subprocess.run([TOOL, "--input"], capture_output=True, text=True)
    assert r.returncode == 1 and "Usage" in r.stderr


def test_text_to_compile_string_interop(tmp_path):
    # the point of att2lfst's shift: a byte-tokenized OpenFst asset then matches
    # fst_compile_string's byte + 1 labels (compose.golden: a -> c)
    src = os.path.join(CORPUS, "compose.input2.att")
    rhs = F.Fst.load_att(src)
    arcs = rhs.arcs(rhs.start)
    assert arcs and arcs[0][0] == ord("b") + 1 and arcs[0][1] == ord("c") + 1


@pytest.mark.parametrize("kind,T", [(0, 4096), (1, 3000)])
def test_load_save_round_trip(kind, T, tmp_path):
    f = F.Fst.bench_transducer(kind, T, 12)     # > 64 KB: the pinned path when a GPU exists
    p = str(tmp_path / "a.fst")
    f.save(p)
    raw = open(p, "rb").read()
    g = F.Fst.load(p)
    p2 = str(tmp_path / "b.fst")
    g.save(p2)
    assert open(p2, "rb").read() == raw
    assert g.num_states == f.num_states and g.start == f.start
    h = F.Fst.load_any(p)                       # fst_batch_load: same bytes
    p3 = str(tmp_path / "c.fst")
    h.save(p3)
    assert open(p3, "rb").read() == raw


def test_load_rejects_bad_files(tmp_path):
    good = O.freeze(O.compile_string(b"ab"))
    cases = {"short": good[:10], "magic": b"XXXX" + good[4:], "truncated": good[:-8],
             "log_for_fst_load": good[:6] + bytes([1]) + good[7:]}
    for name, data in cases.items():
        p = str(tmp_path / (name + ".fst"))
        open(p, "wb").write(data)
        assert F.lib().fst_load(p.encode()) == F.FST_INVALID_HANDLE, name
    assert F.lib().fst_load(str(tmp_path / "missing.fst").encode()) == F.FST_INVALID_HANDLE
    # fst_batch_load accepts the Log header (weight_type 1), rejects an unknown one
    p = str(tmp_path / "log.fst")
    open(p, "wb").write(cases["log_for_fst_load"])
    assert F.lib().fst_batch_load(p.encode()) != F.FST_INVALID_HANDLE
    open(p, "wb").write(good[:6] + bytes([7]) + good[7:])
    assert F.lib().fst_batch_load(p.encode()) == F.FST_INVALID_HANDLE
