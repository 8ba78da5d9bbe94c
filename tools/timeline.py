#!/usr/bin/env python3
"""Print a rocprofv3 kernel trace as a timeline (ms from the first k_rlc_items / k_sig_items
launch), one line per kernel with its queue and stream: for reading stream overlap.
Usage: tools/timeline.py kt_kernel_trace.csv [first_kernel_substring]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
key = sys.argv[2] if len(sys.argv) > 2 else "_items"
first = next(i for i, r in enumerate(rows) if key in r["Kernel_Name"])
t0 = int(rows[first]["Start_Timestamp"])
for r in rows[first:]:
    if "rocclr" in r["Kernel_Name"]:
        continue
    s = (int(r["Start_Timestamp"]) - t0) / 1e6
    e = (int(r["End_Timestamp"]) - t0) / 1e6
    name = r["Kernel_Name"].replace("void ", "").replace("hbtc::", "")
    print("%8.2f %8.2f %7.2f q%s s%s %s" % (s, e, e - s, r["Queue_Id"], r["Stream_Id"], name[:34]))
