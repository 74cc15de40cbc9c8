"""The last host-entry call of a `rocprofv3 --kernel-trace --memory-copy-trace` run of
scripts/e2e_profile.py as a timeline (ms from the call's first event; events > 20 us).
usage: python scripts/e2e_timeline.py <dir with *_kernel_trace.csv, *_memory_copy_trace.csv>"""
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*_kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K",
                       r.get("Queue_Id", r.get("Stream_Id", "")), r["Kernel_Name"][:44],
                       r.get("Grid_Size_X", r.get("Grid_Size", ""))))
    for f in glob.glob(os.path.join(d, "**", "*_memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "M", "",
                       r.get("Direction", r.get("Operation", ""))[:44], r.get("Bytes", "")))
    ev.sort()
    # the last call: from the last pull-kernel start backwards to the preceding gap > 5 ms
    pulls = [i for i, e in enumerate(ev) if "pull_kernel" in e[4]]
    if not pulls:
        print("no pull kernel in the trace")
        return
    i0 = pulls[-1]
    while i0 > 0 and ev[i0][0] - ev[i0 - 1][1] < 5_000_000:
        i0 -= 1
    t0 = ev[i0][0]
    print("start_ms  dur_ms  kind queue  what  grid/bytes")
    first_pull, last_end = None, 0
    for e in ev[i0:]:
        if e[1] - e[0] < 20_000 and "pull_kernel" not in e[4]:
            continue
        if "pull_kernel" in e[4]:
            first_pull = e[0] if first_pull is None else first_pull
            last_end = max(last_end, e[1])
        print(f"{(e[0] - t0) / 1e6:8.3f} {(e[1] - e[0]) / 1e6:8.3f} {e[2]:>2} {e[3]:>4}  {e[4]:44s} {e[5]}")
    print(f"first pull start -> last pull end: {(last_end - first_pull) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
