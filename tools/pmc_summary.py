#!/usr/bin/env python3
"""rocprofv3 --pmc counter_collection.csv files -> per-kernel JSON summary.

Usage: pmc_summary.py OUT.json DIR [DIR ...]
For every kernel: dispatches, VGPR/AGPR/SGPR counts, scratch bytes per lane, LDS bytes, and the
mean per dispatch of every counter collected in the passes under DIR(s).

The derived figures (and `counters_mean_per_dispatch`) are taken over the FULL-SIZE dispatches only:
those whose grid equals the kernel's largest grid in the pass.  A key set's probe pass or a partial
chunk launches the same kernel on a smaller grid, and averaging it in understates the per-launch
figures (VERDICT r05 Weak 3: 4 dispatches, one of them the 62-ciphertext probe).  The mean over
every dispatch stays in `counters_mean_all_dispatches`.  Derived (when present):
  valu_busy      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES   (both quad-cycles; per-wave VALU issue share)
  hbm_read_bytes = 2 * FETCH_SIZE[KB] * 1024  (gfx950 reports half of wide coalesced reads,
                   MI355X_MICROARCH.md "HBM / rocprofv3")
  hbm_write_bytes= WRITE_SIZE[KB] * 1024
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    out_path, dirs = sys.argv[1], sys.argv[2:]
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [(grid, value)]
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f, newline="") as fh:
                for row in csv.DictReader(fh):
                    k = row["Kernel_Name"].split("(")[0]
                    vals[k][row["Counter_Name"]].append((int(row.get("Grid_Size", 0) or 0),
                                                         float(row["Counter_Value"])))
                    meta.setdefault(k, {
                        "vgpr": int(row.get("VGPR_Count", 0) or 0),
                        "agpr": int(row.get("Accum_VGPR_Count", 0) or 0),
                        "sgpr": int(row.get("SGPR_Count", 0) or 0),
                        "scratch_bytes_per_lane": int(row.get("Scratch_Size", 0) or 0),
                        "lds_bytes": int(row.get("LDS_Block_Size", 0) or 0),
                        "grid": int(row.get("Grid_Size", 0) or 0),
                        "workgroup": int(row.get("Workgroup_Size", 0) or 0),
                    })
    res = {}
    for k, cs in vals.items():
        full_grid = max(g for v in cs.values() for g, _ in v)
        full = {c: [x for g, x in v if g == full_grid] for c, v in cs.items()}
        mean = {c: sum(v) / len(v) for c, v in full.items() if v}
        r = dict(meta[k])
        r["grid"] = full_grid
        r["dispatches"] = max(len(v) for v in cs.values())
        r["full_size_dispatches"] = max(len(v) for v in full.values())
        r["counters_mean_per_dispatch"] = {c: round(m, 3) for c, m in sorted(mean.items())}
        r["counters_mean_all_dispatches"] = {c: round(sum(x for _, x in v) / len(v), 3)
                                             for c, v in sorted(cs.items())}
        if "SQ_ACTIVE_INST_VALU" in mean and mean.get("SQ_WAVE_CYCLES"):
            r["valu_busy"] = round(mean["SQ_ACTIVE_INST_VALU"] / mean["SQ_WAVE_CYCLES"], 4)
        if "SQ_INSTS_VALU" in mean and mean.get("SQ_INSTS_SALU") is not None:
            r["valu_to_salu_insts"] = round(mean["SQ_INSTS_VALU"] / max(1.0, mean["SQ_INSTS_SALU"]), 2)
        if "FETCH_SIZE" in mean:
            r["hbm_read_bytes"] = round(2 * mean["FETCH_SIZE"] * 1024)
        if "WRITE_SIZE" in mean:
            r["hbm_write_bytes"] = round(mean["WRITE_SIZE"] * 1024)
        res[k] = r
    with open(out_path, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    for k in sorted(res, key=lambda k: -res[k]["dispatches"]):
        print(k, {x: res[k].get(x) for x in ("dispatches", "full_size_dispatches", "grid", "vgpr", "scratch_bytes_per_lane",
                                              "valu_busy", "hbm_read_bytes", "hbm_write_bytes")})


if __name__ == "__main__":
    main()
