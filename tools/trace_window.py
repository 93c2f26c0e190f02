"""GPU timeline of a bench run's timed region from a rocprofv3 kernel trace (--kernel-trace --output-format csv).

usage: python tools/trace_window.py <run_kernel_trace.csv> <skip forwards> <timed forwards>
Takes the forward kernels (cross_root / posterior_cov / envelope) in start order, skips the first
<skip> forwards' kernels (warmup, graph uploads), and prints the window of <timed> forwards: its span,
the busy time of each queue, the union busy time, and the idle gaps of the union.
"""
import csv
import sys

path, skip, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
rows = []
for r in csv.DictReader(open(path)):
    name = r["Kernel_Name"]
    if any(k in name for k in ("cross_root_plan_kernel", "posterior_cov_kernel", "envelope_kernel")):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), int(r["Queue_Id"]), name.split("(")[0][:40]))
rows.sort()
win = rows[3 * skip:3 * (skip + n)]
t0, t1 = win[0][0], max(e for _, e, _, _ in win)
print(f"forward kernels in trace: {len(rows)}; window {len(win)} kernels, span {(t1 - t0) / 1e3:.1f} us "
      f"({(t1 - t0) / 1e3 / n:.2f} us per forward)")
for q in sorted({w[2] for w in win}):
    ks = [w for w in win if w[2] == q]
    print(f"  queue {q}: {len(ks)} kernels, first start {(ks[0][0] - t0) / 1e3:.1f} us, last end "
          f"{(max(e for _, e, _, _ in ks) - t0) / 1e3:.1f} us, busy {sum(e - s for s, e, _, _ in ks) / 1e3:.1f} us")
busy, cur_s, cur_e, gaps = 0, None, None, []
for s, e, _, _ in win:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
            gaps.append((cur_e - t0, s - cur_e))
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print(f"  union busy {busy / 1e3:.1f} us; gaps > 1 us: " +
      ", ".join(f"@{g0 / 1e3:.1f}:{g / 1e3:.1f}" for g0, g in gaps if g > 1000))
