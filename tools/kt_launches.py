#!/usr/bin/env python3
"""rocprofv3 --kernel-trace CSV -> kt_launches.csv: one row per launch of every hbtc kernel
(kernel, grid_x, workgroup_x, duration_ns, start_ns), the evidence behind bench.py's
rocprof_avg_ms_per_launch (which averages only the dominant kernel's full-size launches: a key
set's probe pass or a partial chunk is a smaller grid).

Usage: kt_launches.py TRACE_DIR OUT.csv
"""
import csv
import glob
import os
import sys


def main():
    trace_dir, out = sys.argv[1], sys.argv[2]
    files = glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit("no kernel_trace.csv under %s" % trace_dir)
    rows = []
    for f in files:
        with open(f, newline="") as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if "hbtc::" not in name:
                    continue
                short = name.split("(")[0].replace("void ", "")
                rows.append((int(r["Start_Timestamp"]), short, int(r.get("Grid_Size_X") or r.get("Grid_Size") or 0),
                             int(r.get("Workgroup_Size_X") or r.get("Workgroup_Size") or 0),
                             int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    t0 = rows[0][0] if rows else 0
    with open(out, "w", newline="") as fh:
        w = csv.writer(fh)
        w.writerow(["kernel", "grid_x", "workgroup_x", "duration_ns", "start_ns"])
        for s, k, g, wg, d in rows:
            w.writerow([k, g, wg, d, s - t0])


if __name__ == "__main__":
    main()
