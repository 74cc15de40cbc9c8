#!/usr/bin/env python3
"""Per-launch SQ counter summary of one kernel from rocprofv3 --pmc CSVs.

usage: sq_summary.py KERNEL_SUBSTRING STRINGS CSV [CSV ...]
Prints each counter per launch and per string, plus derived utilisations: the SQ_*_CYCLES
and SQ_WAIT/ACTIVE counters are in quad-cycles (x4 = cycles), summed over all waves.
"""
import collections
import csv
import sys


def main():
    kern, strings = sys.argv[1], int(sys.argv[2])
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for p in sys.argv[3:]:
        for r in csv.DictReader(open(p)):
            if kern not in r["Kernel_Name"]:
                continue
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
    per = {k: v / len(disp[k]) for k, v in agg.items()}
    for k in sorted(per):
        print(f"{k:28s} {per[k]:16.4g} per launch {per[k] / strings:12.1f} per string")
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in per:
                print(f"{k:28s} {per[k] / wc:8.3f} of wave-cycles")


if __name__ == "__main__":
    main()
