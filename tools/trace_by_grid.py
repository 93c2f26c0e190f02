"""Kernel durations per (kernel, grid) from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

usage: python tools/trace_by_grid.py <dir with *kernel_trace.csv> [name substring ...]
rocprofv3's --stats summary averages every dispatch of a kernel name; a bench run launches the same kernel at
several shapes (one 128-candidate forward for the diagnostics, G batches per launch in the timed region, the
stress legs), so this splits the average by grid size: the row of the timed region's grid is the one to set
beside the bench line's roofline avg_launch_us.
"""
import csv
import glob
import sys


def main():
    d = sys.argv[1]
    subs = sys.argv[2:] or ["envelope_kernel", "posterior_cov", "cross_"]
    rows = {}
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            if not any(s in n for s in subs):
                continue
            g = int(float(r.get("Grid_Size") or 0)) if r.get("Grid_Size") else int(float(r.get("Grid_Size_X", 0))) * int(
                float(r.get("Grid_Size_Y", 1))) * int(float(r.get("Grid_Size_Z", 1)))
            wg = r.get("Workgroup_Size") or r.get("Workgroup_Size_X")
            t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            rows.setdefault((n.split("(")[0], g, wg), []).append(t)
    print(f"{'avg us':>9} {'min us':>9} {'calls':>6} {'grid':>9} {'wg':>5}  kernel")
    for (n, g, wg), ts in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        ts.sort()
        print(f"{sum(ts) / len(ts):9.2f} {ts[0]:9.2f} {len(ts):6d} {g:9d} {wg!s:>5}  {n[:90]}")


if __name__ == "__main__":
    main()
