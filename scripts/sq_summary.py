#!/usr/bin/env python3
"""Per-launch SQ counter summary of one kernel from rocprofv3 --pmc CSVs.

usage: sq_summary.py KERNEL_SUBSTRING STRINGS CSV [CSV ...] [--json OUT]
Prints each counter per launch and per string, plus derived utilisations: the SQ_*_CYCLES
and SQ_WAIT/ACTIVE counters are in quad-cycles (x4 = cycles), summed over all waves.
"""
import collections
import csv
import sys


def main():
    argv = sys.argv[1:]
    out_json = None
    if "--json" in argv:
        i = argv.index("--json")
        out_json = argv[i + 1]
        del argv[i:i + 2]
    sys.argv = [sys.argv[0]] + argv
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
    if out_json:
        import json
        res = {"kernel": kern, "strings_per_launch": strings,
               "per_string": {k: per[k] / strings for k in sorted(per)},
               "of_wave_cycles": {k: per[k] / wc for k in (
                   "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                   "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS") if k in per and wc}}
        json.dump(res, open(out_json, "w"), indent=1)
    if wc:
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                  "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS"):
            if k in per:
                print(f"{k:28s} {per[k] / wc:8.3f} of wave-cycles")


if __name__ == "__main__":
    main()
