"""Aggregate tools/pmc_passes.sh output into per-kernel, per-launch figures.

usage: python tools/pmc_report.py <outdir> <profiles/tag.json> [profiles/r02/pmc_headline.json]

Per kernel (forward instantiations only) and per bench.py stage (its kernels summed per forward): average
per launch of every counter,
per-wave instruction mix, VALU / MFMA busy fractions and HBM bytes.  Units and
gfx950 corrections (MI355X_MICROARCH.md "HBM", "Per-instruction cycle constants"):
  * FETCH_SIZE / WRITE_SIZE are KiB; FETCH_SIZE reports half the bytes of a
    16-B-per-lane streaming read -> x2 for the read side (an estimate for 8-B loads);
  * SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles (x4);
  * SQ_BUSY_CYCLES counts cycles per SE-sampled SQ (reported raw);
  * SQ_VALU_MFMA_BUSY_CYCLES counts cycles, summed over the SIMDs.
"""
import csv
import glob
import json
import sys

KERNELS = {"cross_root_plan_kernel": "cross_root_kernel", "cross_kfill_kernel": "cross_kfill_kernel",
           "cross_big_kernel": "cross_big_kernel", "cross_big32_kernel": "cross_big32_kernel",
           "posterior_cov_big32_kernel": "posterior_cov_big32_kernel",
           "posterior_cov_blk_kernel": "posterior_cov_blk_kernel", "posterior_cov_reg_kernel": "posterior_cov_reg_kernel",
           "posterior_cov_rec2_kernel": "posterior_cov_rec2_kernel",
           "posterior_cov_kernel": "posterior_cov_kernel", "posterior_cov_wide_kernel": "posterior_cov_wide_kernel",
           "posterior_cov_big_kernel": "posterior_cov_big_kernel", "envelope_kernel": "envelope_kernel"}
# bench.py's stages: the kernels one launch of the timed region runs per stage (large n or many candidates:
# the K(x, X) fill before the cross kernel; large B x N: the 64 x 64 or LDS-staged 64 x 128 covariance
# blocks), summed per launch
STAGES = {"cross_root_kernel": ("cross_root_kernel", "cross_kfill_kernel", "cross_big_kernel", "cross_big32_kernel"),
          "posterior_cov_kernel": ("posterior_cov_kernel", "posterior_cov_wide_kernel", "posterior_cov_big_kernel",
                                   "posterior_cov_big32_kernel", "posterior_cov_blk_kernel", "posterior_cov_reg_kernel",
                                   "posterior_cov_rec2_kernel"),
          "envelope_kernel": ("envelope_kernel",)}
# A stage launches one of its alternatives (the K(x, X) fill goes with either cross kernel); the bench's
# diagnostics also run single-batch forwards, so the timed region's alternative is the one for the largest
# launches: the last listed whose main kernel was dispatched (the big blocks are chosen only for launches with
# at least one block per CU, and fp32 plans never take them).
ALTERNATIVES = {"cross_root_kernel": (("cross_root_kernel", "cross_kfill_kernel"), ("cross_big_kernel", "cross_kfill_kernel"),
                                      ("cross_big32_kernel", "cross_kfill_kernel")),
                "posterior_cov_kernel": (("posterior_cov_kernel",), ("posterior_cov_wide_kernel",),
                                         ("posterior_cov_big_kernel",), ("posterior_cov_big32_kernel",),
                                         ("posterior_cov_blk_kernel",), ("posterior_cov_reg_kernel",),
                                         ("posterior_cov_rec2_kernel",)),
                "envelope_kernel": (("envelope_kernel",),)}


def stage_kernels(st, avg, dur):
    alts = [a for a in ALTERNATIVES[st] if a[0] in avg]
    if not alts:
        return [k for k in ALTERNATIVES[st][0] if k in avg]
    return [k for k in alts[-1] if k in avg]


def _name(kn):
    for k, name in KERNELS.items():
        if k in kn and not (k == "envelope_kernel" and ", true," in kn):
            return name
    return None


def _grid(r):
    if "Grid_Size" in r and r["Grid_Size"]:
        return int(float(r["Grid_Size"]))
    return int(float(r.get("Grid_Size_X") or 0)) * int(float(r.get("Grid_Size_Y") or 1)) * int(
        float(r.get("Grid_Size_Z") or 1))
CLOCK_GHZ = 2.4
SIMDS = 1024


def load(out):
    """Per kernel, the counters of its dispatches of the largest grid (the timed region's launch shape: the
    bench's diagnostics also launch single 128-candidate forwards), averaged per dispatch."""
    rows = {}
    for f in glob.glob(f"{out}/*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = _name(r["Kernel_Name"])
            if name:
                rows.setdefault(name, []).append((_grid(r), r["Counter_Name"], float(r["Counter_Value"])))
    agg = {}
    for name, rs in rows.items():
        gmax = max(g for g, _, _ in rs)
        for g, c, v in rs:
            if g == gmax:
                agg.setdefault(name, {}).setdefault(c, []).append(v)
    return {n: {c: sum(v) / len(v) for c, v in d.items()} for n, d in agg.items()}


def durations(out):
    """Per kernel, the mean duration of its dispatches of the largest grid in the kernel trace."""
    rows = {}
    for f in glob.glob(f"{out}/trace/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = _name(r["Kernel_Name"])
            if name:
                rows.setdefault(name, []).append((_grid(r), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    d = {}
    for name, rs in rows.items():
        gmax = max(g for g, _ in rs)
        v = [t for g, t in rs if g == gmax]
        d[name] = sum(v) / len(v)
    return d


def main():
    out, dst = sys.argv[1], sys.argv[2]
    avg, dur = load(out), durations(out)
    rep = figures(avg, dur)
    sav, sdur = {}, {}
    for st in STAGES:
        for k in stage_kernels(st, avg, dur):
            if k in avg:
                acc = sav.setdefault(st, {})
                for c, v in avg[k].items():
                    acc[c] = acc.get(c, 0.0) + v
                if k in dur:
                    sdur[st] = sdur.get(st, 0.0) + dur[k]
    srep = figures(sav, sdur)
    for st in STAGES:
        if st in srep:
            srep[st]["kernels"] = stage_kernels(st, avg, dur)
    json.dump({"kernels": rep, "stages": srep}, open(dst, "w"), indent=2)
    if len(sys.argv) > 3:  # the per-launch figures bench.py reads (roofline traffic / VALU busy), per stage
        keys = ("hbm_bytes_per_launch", "fetch_bytes_x2", "write_bytes", "valu_busy_simd_cycles",
                "valu_insts_per_wave", "valu_busy_frac", "mfma_busy_frac", "mfma_f64_tflops_from_mops", "avg_us",
                "kernels")
        summ = {n: {k: r[k] for k in keys if k in r} for n, r in srep.items()}
        summ["_source"] = {"passes": out, "report": dst}
        json.dump(summ, open(sys.argv[3], "w"), indent=2)
    print(json.dumps({n: {k: v for k, v in r.items() if k != "counters_per_launch"} for n, r in rep.items()},
                     indent=1))


def figures(avg, dur):
    rep = {}
    for name, c in avg.items():
        w = c.get("SQ_WAVES", 0.0) or 1.0
        r = {"counters_per_launch": c, "avg_us": dur.get(name)}
        r["per_wave"] = {k[3:]: v / w for k, v in c.items() if k.startswith("SQ_INSTS") or k in (
            "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
            "SQ_ACTIVE_INST_LDS")}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            r["hbm_bytes_per_launch"] = (2.0 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) * 1024.0
            r["fetch_bytes_x2"] = 2.0 * c.get("FETCH_SIZE", 0.0) * 1024.0
            r["write_bytes"] = c.get("WRITE_SIZE", 0.0) * 1024.0
        if "SQ_ACTIVE_INST_VALU" in c:
            r["valu_busy_simd_cycles"] = 4.0 * c["SQ_ACTIVE_INST_VALU"]   # summed over waves: SIMD-cycles
        if "SQ_INSTS_VALU" in c:
            r["valu_insts_per_wave"] = c["SQ_INSTS_VALU"] / w
        if dur.get(name):
            simd_cycles = dur[name] * 1e-6 * CLOCK_GHZ * 1e9 * SIMDS
            if "SQ_ACTIVE_INST_VALU" in c:
                r["valu_busy_frac"] = 4.0 * c["SQ_ACTIVE_INST_VALU"] / simd_cycles
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                r["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles
            if "SQ_INSTS_VALU_MFMA_MOPS_F64" in c:
                # MOPS counts 512-flop units per the gfx94x convention (16x16x4 f64 = 2 MOPS)
                r["mfma_f64_tflops_from_mops"] = c["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512 / (dur[name] * 1e-6) / 1e12
        rep[name] = r
    return rep


if __name__ == "__main__":
    main()
