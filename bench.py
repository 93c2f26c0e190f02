"""Discrete-KG throughput on MI355X (BASELINE.json headline metric).

One step = one DiscreteKnowledgeGradient forward over a batch of B candidates
per GPU (the reference's ``forward(X[B,1,d])``, discretekg.py:131-159) at the
headline workload: m=2 outputs, n_train=256, n_disc=1024 (32x32 std grid),
S=16 scalarisations, B=128 candidates per GPU, d=2, fp64.  Inputs and GP state
are resident in HBM before timing.  For N>1 (torchrun, one rank per GPU,
RCCL) each rank evaluates its own 128 candidates (weak scaling) and the
per-candidate KG values of every ``--exchange-every`` steps are all-gathered in
one async RCCL call (double buffered), so every rank ends with the whole batch
of every step.  ``--shard scalarisations`` instead gives every rank the same 128
candidates and its own 16 weight rows (16*N in total) and combines the
per-candidate partial sums with one async RCCL all-reduce per exchange (the
north-star exchange; SURVEY.md §8(e) amortises it over K forward batches,
count = K*B, because one collective costs about as much host and link latency as
a whole 128-candidate forward); ``value`` then counts headline-equivalent evals
(candidates x 16 scalarisations).

Prints one JSON line (rank 0): value = KG-evals/s over all ranks, plus the
roofline of the dominant kernel (HIP-event timed, same stream) and a bounded
CPU baseline of the oracle restatement on the host cores.
"""

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "decoupled-kg_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
FP64_PEAK_TFLOPS = 78.6     # MI355X dense FP64 (vector = matrix), MI355X_MICROARCH.md / SURVEY 8(d)
FP32_MFMA_PEAK_TFLOPS = 157.3  # MI355X dense FP32 matrix
HBM_PEAK_GBS = 8000.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1024)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--workload", default="headline")
    ap.add_argument("--shard", choices=["candidates", "scalarisations"], default="candidates",
                    help="axis of the (candidate x scalarisation) space split over ranks (weak scaling)")
    ap.add_argument("--exchange-every", type=int, default=256,
                    help="forward batches per RCCL exchange (count = K*B fp64 values)")
    ap.add_argument("--target", type=int, default=None, help="target_output_ix (decoupled path); default full")
    ap.add_argument("--precision", choices=["fp64", "fp32"], default="fp64",
                    help="fp32: the contractions in fp32 MFMA (DKG_PLAN_F32; BASELINE configs[4], workload stress32)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--profile-reps", type=int, default=50)
    ap.add_argument("--streams", type=int, default=4,
                    help="forward batches in flight: step k runs on stream k %% streams with its own plan workspace")
    ap.add_argument("--graph", type=int, default=1,
                    help="1 = replay each full exchange period (E forwards over the streams) as one captured HIP graph")
    ap.add_argument("--grad-steps", type=int, default=50, help="timed value+gradient calls (0 = skip)")
    ap.add_argument("--pmc", default=os.path.join(REPO, "profiles", "pmc_headline.json"),
                    help="per-kernel HBM traffic from a rocprofv3 --pmc pass (tools/pmc_summary.py)")
    return ap.parse_args()


def stage_model(w, m, n, N, B, S, d):
    """Algorithmic flops / HBM bytes per launch of each kernel (DESIGN.md 'Roofline')."""
    kev = 3 * d + 8  # flops per kernel evaluation (distance + Matern profile)
    fl_cross = sum(B * nn * (nn + 1) + 2 * B * nn + B * nn * kev for nn in n)
    fl_cov = sum(2 * B * N * nn + B * N * kev for nn in n)
    fl_env = B * S * (N + 1) * (4 * m + 2)
    by_cross = sum(8 * (nn * nn + nn * d + B * nn + B) for nn in n) + 8 * B * d
    by_cov = sum(8 * (B * nn + N * nn + B * N) for nn in n) + 8 * (B + N) * d
    by_env = 8 * (m * (N + B * N + B) + S * m + B)
    return {"cross_root_kernel": (fl_cross, by_cross), "posterior_cov_kernel": (fl_cov, by_cov),
            "envelope_kernel": (fl_env, by_env)}


def survey_model(m, n, N, S, B, d):
    """SURVEY.md 8(d) / BASELINE.md algorithmic cost of one forward of B candidates (fp64):
    F = B * (sum_i [2 n_i^2 + 2 n_i N + (3d+8)(n_i+N+1)] + S (N+1)(5m+1)),
    Bytes = 8 [sum_i (n_i^2 + n_i N + N + n_i d) + N d + B d + S m + B]."""
    f_eval = sum(2 * nn * nn + 2 * nn * N + (3 * d + 8) * (nn + N + 1) for nn in n) + S * (N + 1) * (5 * m + 1)
    by = 8 * (sum(nn * nn + nn * N + N + nn * d for nn in n) + N * d + B * d + S * m + B)
    return f_eval * B, by


def cpu_baseline(model, D, W, X, target, seconds, threads):
    """The oracle's structure-faithful restatement of the reference path on host cores."""
    from oracle.discretekg import calculate_discrete_kg, calculate_discrete_kg_conditioning_on_single_output
    from oracle.gp import ModelList, OutputGP

    torch.set_num_threads(threads)
    om = ModelList([OutputGP(m.train_x, m.train_y, m.lengthscale, m.outputscale, m.noise, m.mean_constant,
                             m.kernel, m.nu, m.y_mean, m.y_std) for m in model.models])
    Xc = X.cpu()

    def one(x):
        if target is None:
            return calculate_discrete_kg(om, x, D, W)
        return calculate_discrete_kg_conditioning_on_single_output(om, x, target, D, W)

    one(Xc[0])  # warm-up (builds the per-model caches, as GPyTorch does on first call)
    t0 = time.perf_counter()
    cnt = 0
    while time.perf_counter() - t0 < seconds or cnt < 4:
        one(Xc[cnt % Xc.shape[0]])
        cnt += 1
    dt = time.perf_counter() - t0
    return {"value": cnt / dt, "unit": "KG-evals/s", "cores": threads, "kind": "port",
            "sample": f"{cnt} forwards cycling over the {Xc.shape[0]} headline candidates (per-candidate loop, "
                      f"dense (N+1)^2 posterior covariance, reference epigraph walk; torch fp64 CPU), "
                      f"{dt:.1f} s"}


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # DKG_BENCH_BACKEND=gloo: rehearsal of the N > 1 path with several ranks on one GPU (not a bench line)
    backend = os.environ.get("DKG_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local %= max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.synthetic import WORKLOADS, make_problem
    from dkg_amd.utils import sample_simplex

    w = WORKLOADS[args.workload]
    model, D, X0, W = make_problem(w)
    X = X0
    if args.shard == "candidates":
        # weak scaling: every rank evaluates its own B candidates (Sobol stream per rank)
        if rank > 0:
            X = torch.quasirandom.SobolEngine(w.d, scramble=True, seed=4 + 1000 * rank).draw(w.B, dtype=torch.double)
        W_local = W
    else:
        # weak scaling: S rows per rank out of S*world (rank 0's rows are the headline W)
        W_all = W if world == 1 else torch.cat([W, sample_simplex(w.m, w.S * (world - 1), qmc=True, seed=99)])
        W_local = W_all[rank * w.S:(rank + 1) * w.S]
    acq = DiscreteKnowledgeGradient(model, D, W_local, target_output_ix=args.target, device=dev,
                                    precision=args.precision)
    plan = acq._plan_for(w.B)
    Xd = X.to(dev).contiguous()
    E = max(1, min(args.exchange_every, args.steps))
    from dkg_amd.dist import BatchExchange
    xchg = BatchExchange(w.B, E, "gather" if args.shard == "candidates" else "reduce", S_local=w.S, device=dev)

    main_s = torch.cuda.current_stream(dev)

    def timed(ns, steps, warmup, graph=False):
        """Warmup + `steps` timed forwards with `ns` forward batches in flight.  Stream i (i = k % ns)
        runs step k through its own plan (own Q_X / cov workspace); a stream waits on the main stream
        whenever a new exchange buffer starts, and the main stream waits on every stream before an
        exchange, so each collective sees completed rows and a row is never rewritten under one."""
        streams = [main_s] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
        plans = [plan] + [acq._state.plan(acq._W, acq.target_output_ix, plan.max_B, f32=args.precision == "fp32")
                          for _ in range(ns - 1)]

        def join():
            for s in streams[1:]:
                main_s.wait_stream(s)

        def step(k):
            kg = xchg.row(k)
            if ns > 1 and k % E == 0:
                for s in streams[1:]:
                    s.wait_stream(main_s)
            with torch.cuda.stream(streams[k % ns]):
                plans[k % ns].forward_into(Xd, kg)
            if k % E == E - 1:
                join()
            xchg.done(k)

        for k in range(warmup):
            step(k)
        join()
        xchg.flush(warmup)
        torch.cuda.synchronize()

        graphs = []
        if graph and steps >= E:
            # one graph per exchange buffer: the E forwards of a period, forked over the streams exactly
            # as the eager path does; replayed on the main stream, so the collective after it orders as before
            for slot in range(2):
                g = torch.cuda.CUDAGraph()
                # thread_local: the RCCL watchdog thread may query events while this thread captures
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    cs = torch.cuda.current_stream(dev)
                    lanes = [cs] + streams[1:]
                    for s in lanes[1:]:
                        s.wait_stream(cs)
                    for r in range(E):
                        with torch.cuda.stream(lanes[r % ns]):
                            plans[r % ns].forward_into(Xd, xchg.bufs[slot][r])
                    for s in lanes[1:]:
                        cs.wait_stream(s)
                graphs.append(g)
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record()
        for s in streams[1:]:
            s.wait_stream(main_s)
        k0 = 0
        if graphs:
            while k0 + E <= steps:
                xchg.row(k0)
                graphs[(k0 // E) % 2].replay()
                xchg.done(k0 + E - 1)
                k0 += E
        for k in range(k0, steps):
            step(k)
        join()
        xchg.flush(steps)
        ev1.record()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        gpu_s = ev0.elapsed_time(ev1) / 1e3
        t = torch.tensor([max(wall, gpu_s)], dtype=torch.double, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    single = None
    if args.streams > 1 or args.graph:
        e1 = timed(1, args.steps, args.warmup)
        single = {"value": world * w.B * args.steps / e1, "ms_per_step": e1 / args.steps * 1e3}
    elapsed = timed(max(1, args.streams), args.steps, args.warmup, graph=bool(args.graph))
    value = world * w.B * args.steps / elapsed

    # ---- per-kernel durations (HIP events on the launch stream), roofline of the dominant kernel
    names = ["cross_root_kernel", "posterior_cov_kernel", "envelope_kernel"]
    avg_ms = [plan.time_stage(Xd, k, args.profile_reps) for k in range(3)]
    model_fb = stage_model(w, w.m, [mm.num_train for mm in model.models], D.shape[0], w.B, w.S, w.d)
    dom = max(range(3), key=lambda i: avg_ms[i])
    fl, by = model_fb[names[dom]]
    # every stage is fp64-compute bound (DESIGN.md "Roofline"): MFMA for cross/cov, fp64 VALU (same 78.6 TF
    # peak) for the envelope; HBM bytes per launch are << peak*duration for all three.
    peak = FP32_MFMA_PEAK_TFLOPS if (args.precision == "fp32" and dom < 2) else FP64_PEAK_TFLOPS
    bound, ach, unit = "mfma", fl / (avg_ms[dom] * 1e-3) / 1e12, "TFLOP/s"
    traffic = None
    if os.path.exists(args.pmc):
        try:
            traffic = json.load(open(args.pmc)).get(names[dom], {}).get("hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    roof = {"kernel": names[dom], "bound": bound, "achieved": ach, "peak": peak, "unit": unit,
            "frac": ach / peak, "traffic": traffic, "algorithmic_flops": fl, "algorithmic_bytes": by,
            "avg_launch_us": avg_ms[dom] * 1e3,
            "stages_us": {n: a * 1e3 for n, a in zip(names, avg_ms)}}

    # ---- whole-forward roofline as BASELINE.md defines it: max(F/P, Bytes/BW) / T_measured
    f_fwd, b_fwd = survey_model(w.m, [mm.num_train for mm in model.models], D.shape[0], w.S, w.B, w.d)
    t_fwd = elapsed / args.steps
    t_min = max(f_fwd / (FP64_PEAK_TFLOPS * 1e12), b_fwd / (HBM_PEAK_GBS * 1e9))
    fwd_roof = {"definition": "BASELINE.md: max(F/P_fp64, Bytes/BW_HBM) / T_forward", "flops": f_fwd,
                "bytes": b_fwd, "t_min_us": t_min * 1e6, "t_forward_us": t_fwd * 1e6, "frac": t_min / t_fwd}

    # ---- SURVEY.md 8(d) diagnostics of the batch: short-circuit rate, KG distribution, envelope sizes
    kg_s, pairs_s, hull_s = plan.forward_stats(Xd)
    pairs_c, hull_c, kg_c = pairs_s.cpu(), hull_s.cpu().long(), kg_s.cpu()
    hist = torch.bincount(hull_c.reshape(-1)).tolist()
    pair_stats = {"pairs": int(pairs_c.numel()),
                  "short_circuit_frac": float((hull_c == 1).double().mean()),
                  "zero_kg_frac": float((pairs_c == 0).double().mean()),
                  "envelope_lines_mean": float(hull_c.double().mean()),
                  "envelope_lines_hist": {str(h): c for h, c in enumerate(hist) if c},
                  "kg_quantiles": {str(q): float(torch.quantile(kg_c, q)) for q in (0.0, 0.1, 0.5, 0.9, 1.0)}}

    # ---- value + gradient (dkg_plan_forward_grad: the optimize_acqf L-BFGS-B path), same batch
    grad_info = None
    if args.grad_steps > 0 and args.precision == "fp64":
        gplan = acq._plan_for(w.B, grad=True)
        for _ in range(3):
            gplan.forward_grad(Xd)
        torch.cuda.synchronize()
        g0 = time.perf_counter()
        for _ in range(args.grad_steps):
            gplan.forward_grad(Xd)
        torch.cuda.synchronize()
        gdt = (time.perf_counter() - g0) / args.grad_steps
        grad_info = {"value": w.B / gdt, "unit": "KG-evals+gradients/s (per GPU)", "ms_per_step": gdt * 1e3}

    out = None
    if rank == 0:
        cpu = None
        if args.cpu_seconds > 0 and world == 1:
            cpu = cpu_baseline(model, D, W, X0, args.target, args.cpu_seconds, args.cpu_threads)
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "KG-evals/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64" if args.precision == "fp64" else "f32 contractions / f64 envelope",
            "data": f"synthetic: seeded GP-prior draw, lengthscales family ({w.lengthscales}, s={w.outputscales}, "
                    f"noise {'%g x s' % w.noise_rel if w.noise_rel > 0 else w.noise})",
            "config": {"workload": args.workload, "m": w.m, "n_train": w.n_train, "n_disc": D.shape[0],
                       "S": w.S, "B_per_gpu": w.B, "d": w.d,
                       "path": "full" if args.target is None else f"target_output_ix={args.target}",
                       "shard": args.shard,
                       "parallelism": f"{args.shard} sharded over {world} GPU(s); one async RCCL "
                                      f"{'all-gather' if args.shard == 'candidates' else 'all-reduce'} "
                                      f"per {E} forward batches",
                       "exchange_every": E, "streams": max(1, args.streams),
                       "hip_graph": bool(args.graph)},
            "single_stream": single,
            "forward_calls_per_s": world * args.steps / elapsed,
            "value_and_grad": grad_info,
            "roofline": roof,
            "forward_roofline": fwd_roof,
            "batch_stats": pair_stats,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
