"""Symbolizes the CPU samples of libfst_amd/concurrent_calls (CC_PROF=<file>): prints the
hottest leaf functions and, for each, its most common callers (addr2line on the objects
the samples name, which are the same files in this container and on the GPU box).
usage: python scripts/ccprof_report.py <samples> [--top N]"""
import collections
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local(path):
    if "/libfst_amd/" in path and not os.path.exists(path):  # the box's repo root
        return os.path.join(REPO, "libfst_amd", path.split("/libfst_amd/", 1)[1])
    return path


def main():
    top = int(sys.argv[sys.argv.index("--top") + 1]) if "--top" in sys.argv else 12
    samples = [line.split() for line in open(sys.argv[1]) if line.strip()]
    need = collections.defaultdict(set)
    for fr in samples:
        for x in fr:
            obj, off = x.rsplit(":", 1)
            need[obj].add(off)
    name = {}
    for obj, offs in need.items():
        offs = sorted(offs)
        p = local(obj)
        if not os.path.exists(p):
            for o in offs:
                name[(obj, o)] = f"{os.path.basename(obj)}+{o}"
            continue
        out = subprocess.run(["addr2line", "-f", "-C", "-e", p] + offs, capture_output=True,
                             text=True).stdout.splitlines()
        for i, o in enumerate(offs):
            fn = out[2 * i] if 2 * i < len(out) else "??"
            name[(obj, o)] = f"{fn} [{os.path.basename(obj)}]" if fn != "??" else \
                f"{os.path.basename(obj)}+{o}"
    sym = [[name[tuple(x.rsplit(":", 1))] for x in fr] for fr in samples]
    leaf = collections.Counter(s[0] for s in sym)
    print(f"{len(sym)} samples")
    for fn, n in leaf.most_common(top):
        print(f"{n:6d} {100.0 * n / len(sym):5.1f}%  {fn}")
        chains = collections.Counter(" <- ".join(s[1:6]) for s in sym if s[0] == fn)
        for ch, m in chains.most_common(3):
            print(f"           {m:5d}  <- {ch[:300]}")


if __name__ == "__main__":
    main()
