#!/usr/bin/env python
"""Benchmark: Goku z=0 P(k) 1128LF/36HF multi-bin GPR on MI355X.

Metric (BASELINE.json): LML evals/sec + train+predict wall-clock, Goku multi-bin.

  step      = one MultiFidelityGPModel.optimize(use_adam=True) iteration on the
              Goku training set: LML value + analytic gradient + Keras-Adam update
              (mfgpflow/linear.py:203-214), executed by libmfgp.so from a hipGraph.
  value     = LML value+grad evaluations per second, whole job.  With N GPUs the
              64 k-bins are sharded into N contiguous blocks, one independent
              per-shard-theta emulator per rank (SURVEY §8(e) "embarrassing mode",
              north_star: bins shard with no inner-loop collective): every rank
              completes one evaluation of its block's model per step, so
              value = N * steps / max-over-ranks time ("scaling": "weak": each GPU
              runs one Gram + Cholesky + its bins' solves per step; the Gram and
              Cholesky dominate and do not shrink with N).  bin_throughput
              (k-bins processed per second, = 64 * steps / time) is reported beside
              it: it stays ~flat in N for the same reason.
  inputs    = rank 0 reads the reference's Goku txt files (tests/golden/data) and
              RCCL-broadcasts them once; no collective inside the timed loop.
  extras    = train_predict_s: the notebook protocol optimize(1000, lr=0.1) +
              predict_f(X_test) wall-clock of a fresh model, after one untimed predict_f
              (per-process kernel loading) (max over ranks); roofline of the
              dominant kernel family from live hipEvent phase times; cpu_baseline:
              the fp64 oracle (oracle/mfgp_oracle.py) timed on this host (rank 0, N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

GOKU = os.path.join(ROOT, "tests", "golden", "data", "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0")
FP64_PEAK_TFLOPS = 78.6   # MI355X dense FP64 (vector = matrix on gfx950), MI355X_MICROARCH.md
FP32_PEAK_TFLOPS = 157.3  # MI355X dense FP32 (v_mfma_f32_32x32x2_f32 = the f32 vector rate), MI355X_MICROARCH.md
HBM_PEAK_GBS = 8000.0
# HBM bytes per dispatch from the committed rocprofv3 PMC passes (tools/profile_round.sh ->
# tools/summarize_profile.py); the bench cannot count PMC on itself.
def latest_pmc_summary(config="goku"):
    """profiles/rNN/<config>/pmc_summary.json (or round 1's profiles/r01/pmc_summary.json for Goku) of
    the latest round that has one."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", config, "pmc_summary.json")))
    if not found and config == "goku":
        found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "pmc_summary.json")))
    return found[-1] if found else None


def _pmc_entry(kernel_prefix, nb, config):
    path = latest_pmc_summary(config)
    try:
        with open(path) as f:
            kern = json.load(f)["kernels"]
    except (TypeError, OSError, ValueError, KeyError):
        return None, None
    for name, v in kern.items():
        if f"{kernel_prefix}<{nb}>" in name or f"{kernel_prefix}(" in name:
            return v, os.path.relpath(path, ROOT)
    return None, None


def pmc_traffic(kernel_prefix, nb, config="goku"):
    """(bytes per dispatch, source) of the dominant kernel from the committed PMC summary."""
    v, src = _pmc_entry(kernel_prefix, nb, config)
    return (v["hbm_bytes"], src) if v else (None, None)


def rocprof_avg_us(kernel_prefix, nb, config="goku"):
    """(average launch duration in us, source) of a kernel from the committed rocprofv3 kernel
    trace of this config (the summary's avg_duration_ns, taken from kernel_stats.csv)."""
    v, src = _pmc_entry(kernel_prefix, nb, config)
    if not v or not v.get("avg_duration_ns"):
        return None, None
    return v["avg_duration_ns"] * 1e-3, src


def pmc_step_traffic(config, step_kernel):
    """(HBM bytes per step, source): every kernel's mean bytes per dispatch x its dispatches per
    dispatch of step_kernel (one per step), from the committed PMC summary."""
    path = latest_pmc_summary(config)
    try:
        with open(path) as f:
            kern = json.load(f)["kernels"]
    except (TypeError, OSError, ValueError, KeyError):
        return None, None
    steps = next((v["dispatches"] for n, v in kern.items() if n.startswith(step_kernel)), 0)
    if not steps:
        return None, None
    return int(sum(v["hbm_bytes"] * v["dispatches"] for v in kern.values()) / steps), os.path.relpath(path, ROOT)


def load_goku():
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    ps = PowerSpecs()
    ps.read_from_txt(GOKU)
    return multifidelity_training_set(ps)


def bcast_label(world):
    """How the inputs reached this rank (the `data` field of the JSON line)."""
    if world == 1:
        return "read on the one rank"
    backend = os.environ.get("MFGP_DIST_BACKEND", "nccl")
    return ("RCCL" if backend == "nccl" else backend) + "-broadcast from rank 0"


def broadcast_inputs(rank, world, device):
    """Rank 0 reads the txt files; one RCCL broadcast of the packed inputs."""
    from multi_fidelity_gpflow_amd.distributed import broadcast_arrays
    arrays = list(load_goku()) if rank == 0 else None
    return broadcast_arrays(arrays, rank, world, device)


def make_model(X, Yr, dtype=None):
    import multi_fidelity_gpflow_amd as M
    d = X.shape[1] - 1
    return M.MultiFidelityGPModel(X, Yr, M.SquaredExponential(lengthscales=np.ones(d), variance=1.0),
                                  M.SquaredExponential(lengthscales=np.ones(d), variance=1.0), dtype=dtype)


def step_flops(n, p, d):
    """one LML value+grad evaluation (fp64)."""
    gram = (n * (n + 1) / 2) * (3 * d + 6)
    return gram + n ** 3 / 3 + n * n * p + 2 * n ** 3 / 3 + 2 * n * n * p + n * (n + 1) / 2 * (4 * d + 10)


def roofline(model, n, p, d, reps=10, pmc=True):
    """Dominant kernel family from live hipEvent phase times (launch stream)."""
    from multi_fidelity_gpflow_amd.engine import gpr_phase_times
    eng, X, Y = model._device_data()
    theta = torch.tensor(model._theta_map().theta(), dtype=torch.float64, device=eng.device)
    gpr_phase_times(eng, X, Y, theta)   # warm
    acc = np.zeros(5)
    for _ in range(reps):
        acc += np.array(gpr_phase_times(eng, X, Y, theta))
    ms = acc / reps
    names = ["pre", "gram", "chol_steps", "grad", "finalize"]
    nb = eng.tile()
    T = -(-n // nb)
    # algorithmic work per phase (SURVEY §8(d) figures)
    flops = {
        "gram": (n * (n + 1) / 2) * (3 * d + 6),
        # potrf + L^{-1} (trtri) + Z = L^{-1} Y + alpha = L^{-T} Z (fused into the steps)
        "chol_steps": n ** 3 / 3 + n ** 3 / 3 + n * n * p + n * n * p,
        "grad": n ** 3 / 3 + n * n * p + n * (n + 1) / 2 * (4 * d + 10),
    }
    flow = eng.flow_runs(n)    # one persistent k_chol_flow launch, else T k_chol_step launches
    launches = {"gram": 1, "chol_steps": 1 if flow else T, "grad": 1}
    dom = max(flops, key=lambda k: ms[names.index(k)])
    t_ms = ms[names.index(dom)]
    per_launch_ms = t_ms / launches[dom]
    per_launch_flop = flops[dom] / launches[dom]
    achieved = per_launch_flop / (per_launch_ms * 1e-3) / 1e12
    kname = {"chol_steps": "k_chol_flow" if flow else "k_chol_step", "gram": "k_gram", "grad": "k_grad"}[dom]
    traffic, tsrc = pmc_traffic(kname, nb) if pmc else (None, None)
    # headline achieved / frac from the committed rocprofv3 average of the same kernel (VERDICT r5
    # #9); the live hipEvent figure (an eager evaluation, launch stream) beside it
    rp_us, rp_src = rocprof_avg_us(kname, nb) if pmc else (None, None)
    achieved_rp = per_launch_flop / (rp_us * 1e-6) / 1e12 if rp_us else None
    head = achieved_rp if achieved_rp is not None else achieved
    return {
        "kernel": kname,
        "bound": "mfma",
        "achieved": round(head, 4),
        "achieved_source": (f"algorithmic flop per launch / rocprofv3 average {rp_us:.1f} us ({rp_src})"
                            if achieved_rp is not None else "algorithmic flop per launch / live hipEvent time"),
        "peak": FP64_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(head / FP64_PEAK_TFLOPS, 5),
        "achieved_live": round(achieved, 4),
        "frac_live": round(achieved / FP64_PEAK_TFLOPS, 5),
        "traffic": traffic,
        "traffic_unit": "bytes per launch (FETCH_SIZE x2 + WRITE_SIZE)",
        "traffic_source": tsrc,
        "launches_per_step": launches[dom],
        "avg_launch_us": round(per_launch_ms * 1e3, 3),
        "flop_per_launch": per_launch_flop,
        "phase_ms": {k: round(float(v), 4) for k, v in zip(names, ms)},
    }


def roofline_f32(model, reps=3, pmc=True):
    """fp32 path: hipEvents around every launch of one value+grad evaluation (serial schedule,
    launch stream), summed per phase.  The dominant kernel is the tile update k32_update (the
    in-panel updates, K = 128, and the trailing updates, K = 128 * panel); achieved = the tile
    flops its launches perform (all but the strictly upper half of the diagonal tiles) / their
    summed launch time; traffic = the committed PMC mean bytes per k32_update dispatch x its
    launches per step."""
    from multi_fidelity_gpflow_amd.engine import gpr_phase_times_ex
    eng, X, Y = model._device_data()
    theta = torch.tensor(model._theta_map().theta(), dtype=torch.float64, device=eng.device)
    gpr_phase_times_ex(eng, X, Y, theta)   # warm
    acc = {}
    for _ in range(reps):
        for k, (ms, fl, la) in gpr_phase_times_ex(eng, X, Y, theta).items():
            a = acc.setdefault(k, [0.0, fl, la])
            a[0] += ms / reps
    kn = {"update_out": "k32_update", "update_in": "k32_update", "grad": "k32_grad", "diag": "k32_diag",
          "panel": "k32_panel", "gram": "k32_gram", "alpha": "k32_alpha", "finalize": "k32_zsum"}
    per_kernel = {}
    for k, (ms_, fl_, la_) in acc.items():
        e = per_kernel.setdefault(kn[k], [0.0, 0.0, 0])
        e[0] += ms_
        e[1] += fl_
        e[2] += la_
    kname = max(per_kernel, key=lambda k: per_kernel[k][0])
    ms, fl, la = per_kernel[kname]
    achieved = fl / (ms * 1e-3) / 1e12
    traffic, tsrc = pmc_traffic(kname, 0, "synth") if pmc else (None, None)
    if traffic is not None:
        traffic = int(traffic * la)
    return {
        "kernel": kname + (" (in-panel K = 128 and trailing K = 128 x panel tile updates)"
                           if kname == "k32_update" else ""),
        "bound": "mfma",
        "achieved": round(achieved, 3),
        "peak": FP32_PEAK_TFLOPS,
        "unit": "TFLOP/s",
        "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
        "traffic": traffic,
        "traffic_unit": "bytes per step summed over the kernel's launches (FETCH_SIZE x2 + WRITE_SIZE)",
        "traffic_source": tsrc,
        "launches_per_step": la,
        "avg_launch_us": round(ms * 1e3 / max(la, 1), 3),
        "flop_per_launch": fl / max(la, 1),
        "phase_ms": {k: round(v[0], 4) for k, v in acc.items()},
        "phase_tflops": {k: round(v[1] / (v[0] * 1e-3) / 1e12, 2) if v[0] > 0 and v[1] > 0 else None
                         for k, v in acc.items()},
        "phase_launches": {k: v[2] for k, v in acc.items()},
        "serial_sum_ms": round(sum(v[0] for v in acc.values()), 3),
    }


def _median_rate(fn, min_evals=20, budget_s=6.0):
    """evals/s from the median of >= min_evals timed calls after one warm-up,
    stopping early at budget_s once min_evals are in (or after 3 if one call is that slow)."""
    fn()
    ts = []
    t_start = time.perf_counter()
    while len(ts) < min_evals:
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s and len(ts) >= 3:
            break
    return 1.0 / float(np.median(ts)), len(ts)


def host_cpus():
    """(cores this process may run on, how that was found): the CPU affinity mask, capped by the
    cgroup CPU quota when one is set (a container's share of a large host)."""
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = os.cpu_count() or 1
    src = f"sched_getaffinity {aff}"
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            q = max(1, int(int(quota) // int(period)))
            src += f", cgroup cpu.max quota {q}"
            aff = min(aff, q)
    except (OSError, ValueError):
        pass
    return aff, src


def cpu_protocol_measured():
    """The CPU baseline's full protocol (1000 Adam steps + predict_f on the box's cores), timed once
    by tools/cpu_protocol.py into profiles/rNN/cpu_protocol.json (the latest round that has one)."""
    import glob
    found = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]", "cpu_protocol.json")))
    if not found:
        return None
    try:
        with open(found[-1]) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None
    return {"train_predict_s": d.get("train_predict_s"), "steps": d.get("steps"), "cores": d.get("cores"),
            "source": os.path.relpath(found[-1], ROOT) + " (tools/cpu_protocol.py, timed once on a GPU box host)"}


def cpu_baseline(X, Y):
    """fp64 torch-CPU restatement of the reference path (oracle/torch_oracle.py, checked against
    the KAT-pinned oracle/mfgp_oracle.py) on this host: all threads and 1 thread, value-only and
    value+grad.  Bounded sample: <= ~6 s of CPU work per leg."""
    from oracle import torch_oracle as TO
    Xt = torch.as_tensor(X, dtype=torch.float64)
    Yt = torch.as_tensor(Y, dtype=torch.float64)
    args = TO.initial_args(X.shape[1] - 1)
    torch_threads = torch.get_num_threads()
    nthreads, cores_src = host_cpus()
    legs = {}
    for label, threads in (("all", nthreads), ("one", 1)):
        torch.set_num_threads(threads)
        try:
            vg, nvg = _median_rate(lambda: TO.lml_and_grad(Xt, Yt, *args))
            v, nv = _median_rate(lambda: TO.lml(Xt, Yt, *args))
        finally:
            torch.set_num_threads(torch_threads)
        legs[label] = {"threads": threads, "value_grad_evals_s": round(vg, 3), "value_evals_s": round(v, 3),
                       "samples": [nvg, nv]}
    return {"value": legs["all"]["value_grad_evals_s"], "unit": "LML value+grad evals/s",
            "cores": nthreads, "kind": "port", "nproc": os.cpu_count(), "cores_source": cores_src,
            "torch_default_threads": torch_threads,
            "value_only_evals_s": legs["all"]["value_evals_s"],
            "one_core": legs["one"],
            "train_1000_adam_s_est": round(1000.0 / legs["all"]["value_grad_evals_s"], 2),
            "protocol_measured": cpu_protocol_measured(),
            "sample": (f"Goku (N={X.shape[0]}, P={Y.shape[1]}) fp64 LML value+grad and value-only evaluations at "
                       f"the initial theta, oracle/torch_oracle.py (MKL Cholesky/TRSM/GEMM), median of >=20 "
                       f"after warm-up (fewer if a leg exceeds ~6 s), torch threads {nthreads} (the cores available: "
                       f"{cores_src}) and 1; "
                       f"train_1000_adam_s_est = 1000 / value")}


def svgp_elbo_flops(n, m, L, p, d):
    """one SVGP ELBO evaluation L[(M(M+1)/2 + MN)(3D+6) + M^3/3 + 2M^2 N] + 4NLP."""
    return L * ((m * (m + 1) / 2 + m * n) * (3 * d + 6) + m ** 3 / 3 + 2 * m * m * n) + 4 * n * L * p


def svgp_step_mfma_flops(n, m, L, nb=32):
    """Executed f64 MFMA flops of one SVGP optimize() step on the padded NB-tiles (2 NB^3 per tile
    product), forward and reverse pass, per the launch sequence of mfgp_svgp.hip / mfgp_svgp_grad.hip:
      forward  Kuu factor (blocked Cholesky + inverse, ~Tm^3/3 + Tm^3/6 tile products),
               A = Li Kuf and B = Lq^T A (the gradient pass's two triangular GEMMs: Tn Tm(Tm+1)/2
               each; the value-only path's fused k_svgp_cond2 forms B = C Kuf with C = Lq^T Li);
      reverse  gA (Tn Tm(Tm+1)/2), dE/dLi (tril, Tn Tm(Tm+1)/2), Gb Li^T (sum min(i, j) + 1),
               Psi Li and Li^T (.) (Tm^2(Tm+1)/2 each), dE/dKuf (Tn Tm(Tm+1)/2),
               dE/dLq (tril, Tn Tm(Tm+1)/2)."""
    Tm, Tn = -(-m // nb), -(-n // nb)
    tri = Tm * (Tm + 1) // 2
    fwd = Tm ** 3 / 3 + Tm ** 3 / 6 + 2 * Tn * tri
    rev = 4 * Tn * tri + sum(min(i, j) + 1 for i in range(Tm) for j in range(Tm)) + 2 * Tm * tri
    return L * (fwd + rev) * 2 * nb ** 3


def svgp_leg(X, Yr, Xt, steps, warmup, world=1, device=None, train_predict=True, latent=True):
    """BASELINE configs[3]: the Goku SVGP models of notebooks/demo: goku power spectra.ipynb --
    SingleBinSVGP (M=300 KMeans centres, L=P=64; cell 10, 1000 iterations, published 2237.47 s on
    the M1) and LatentMFCoregionalizationSVGP (L=15, M=300; published 1020.22 s for 2000).  A step
    is one optimize() iteration: ELBO + analytic gradient + Keras Adam with the CosineDecay
    schedule, replayed from hipGraphs (graphs captured in warm-up).  N > 1: each rank trains the
    single-bin model of its own bin block (per-shard Z / noise, no collective).  Returns the
    per-rank times and the line's fields."""
    import multi_fidelity_gpflow_amd as M
    n, d = X.shape[0], X.shape[1] - 1
    pr = Yr.shape[1]
    K, W = steps, warmup
    kern = lambda: M.SquaredExponential(lengthscales=np.ones(d))

    def timed(model, max_iters):
        tr = M.svgp._SVGPTrainer(model, (X, Yr), max_iters=max_iters, initial_lr=0.1, graph=True, graph_chunk=10)
        tr.run(W)
        with torch.cuda.stream(tr.stream):
            tr.runner.prepare(K)   # capture every graph the timed run replays
        tr.sync()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        tr.run(K)
        tr.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        tr.close()
        return dt

    sb = M.SingleBinSVGP(X, Yr, kern(), kern(), pr, Z=np.zeros((300, d + 1)))
    dt_sb = timed(sb, K + W)
    dt_lat = None
    if latent:
        lat = M.LatentMFCoregionalizationSVGP(X, Yr, kern(), kern(), num_latents=min(15, pr), num_inducing=300,
                                              num_outputs=pr, w_type="diagonal", window_fraction=0.4, scale=0.2)
        dt_lat = timed(lat, max(K + W, 2000))
    # notebook protocol for the single-bin model: a fresh model, optimize(max_iters=1000, initial_lr=0.1)
    train_s = None
    if train_predict:
        m2 = M.SingleBinSVGP(X, Yr, kern(), kern(), pr, Z=np.zeros((300, d + 1)))
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        m2.optimize((X, Yr), max_iters=1000, initial_lr=0.1, unfix_noise_after=500)
        m2.predict_f(Xt)
        torch.cuda.synchronize()
        train_s = time.perf_counter() - t1
    fl = svgp_elbo_flops(n, 300, pr, pr, d)
    achieved = fl * K / dt_sb / 1e12
    fx = svgp_step_mfma_flops(n, 300, pr)
    executed = fx * K / dt_sb / 1e12
    tb, tsrc = pmc_step_traffic("goku_svgp", "mfgp::k_adam_packed")
    return {
        "steps": K, "warmup": W,
        "ms_per_step": round(dt_sb / K * 1e3, 4),
        "iters_per_s": round(world * K / dt_sb, 3),
        "config": {"workload": "goku_singlebin_svgp_step", "n": n, "d": d, "m": 300, "latents": pr,
                   "bins_per_rank": pr},
        "latent_l15": None if dt_lat is None else {
            "latents": min(15, pr), "ms_per_step": round(dt_lat / K * 1e3, 4),
            "iters_per_s": round(world * K / dt_lat, 3), "published_m1_s_per_iter": round(1020.22 / 2000, 4)},
        "train_1000_predict_s": None if train_s is None else round(train_s, 3),
        "published_m1": {"train_1000_s": 2237.47, "source": "notebooks/demo: goku power spectra.ipynb:451"},
        "roofline": {"kernel": "whole optimize() iteration (SURVEY §8(d) ELBO-value flops only; the gradient's "
                               "reverse pass is not counted, so this is a lower bound)",
                     "bound": "mfma", "achieved": round(achieved, 4), "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(achieved / FP64_PEAK_TFLOPS, 5), "traffic": tb,
                     "traffic_unit": "HBM bytes per optimize() iteration (FETCH_SIZE x2 + WRITE_SIZE, every "
                                     "kernel, single-bin model)",
                     "traffic_source": tsrc,
                     "traffic_gbs": None if tb is None else round(tb / (dt_sb / K) / 1e9, 1),
                     "flop_per_step": fl,
                     "executed": {"what": "f64 MFMA tile flops issued by the forward and reverse pass "
                                          "(padded NB = 32 tiles; svgp_step_mfma_flops)",
                                  "flop_per_step": fx, "achieved": round(executed, 4),
                                  "frac": round(executed / FP64_PEAK_TFLOPS, 5)}},
    }


def bench_svgp(args):
    """--config goku_svgp: the SVGP leg as the headline line."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = dist_device_index()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        init_dist(device)
    X, Y, Xt, Yt = broadcast_inputs(rank, world, device)
    from multi_fidelity_gpflow_amd.distributed import bin_block
    b0, b1 = bin_block(Y.shape[1], rank, world)
    Yr = np.ascontiguousarray(Y[:, b0:b1])
    leg = svgp_leg(X, Yr, Xt, args.steps, args.warmup, world, device, train_predict=not args.no_train_predict,
                   latent=not args.no_latent)
    shared = shared_inducing_leg(X, Yr, min(args.steps, 50), min(args.warmup, 5), rank, world, device) \
        if world > 1 else None
    if rank == 0:
        cfg = dict(leg.pop("config"), parallelism=f"bins{world}" if world > 1 else "single")
        line = {
            "metric": "SVGP optimize iterations/s (Goku SingleBinSVGP M=300, L=P=64: ELBO + gradient + Adam)",
            "value": leg.pop("iters_per_s"), "unit": "iters/s", "n_gpus": world, "steps": leg.pop("steps"),
            "warmup": leg.pop("warmup"), "ms_per_step": leg.pop("ms_per_step"), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f64",
            "data": "Goku z=0 P(k) (reference data files, tests/golden/data), " + bcast_label(world),
            "config": cfg,
        }
        line.update(leg)
        if shared is not None:
            line["shared_inducing"] = shared
        line["cpu_baseline"] = None
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()
    return 0


def shared_inducing_leg(X, Yr, steps, warmup, rank, world, device):
    """N > 1: the reference's ONE SingleBinSVGP over all bins (singlebin_svgp.py:39-62): each rank
    its bin block's per-bin state, Z (rank 0's KMeans centres) and the noise shared and trained,
    one all-reduce of M (D+1) + 5 doubles per step (distributed.SharedInducingTrainer).  value =
    model iterations / s (strong scaling)."""
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.distributed import SharedInducingTrainer, broadcast_inducing
    d = X.shape[1] - 1
    kern = lambda: M.SquaredExponential(lengthscales=np.ones(d))
    model = broadcast_inducing(M.SingleBinSVGP(X, Yr, kern(), kern(), Yr.shape[1], Z=np.zeros((300, d + 1))),
                               rank, world, device)
    tr = SharedInducingTrainer(model, (X, Yr), steps + warmup, 0.1)
    tr.run(warmup)
    tr.sync()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    tr.run(steps)
    tr.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    tr.finish()
    return {"mode": "shared_inducing", "scaling": "strong", "steps": steps, "warmup": warmup,
            "ms_per_step": round(dt / steps * 1e3, 4), "value": round(steps / dt, 3), "unit": "iters/s",
            "collective": f"one all-reduce of {model.inducing_variable.numpy().size + 5} doubles per step"}


HBS = os.path.join(ROOT, "tests", "golden", "data", "50_LR_3_HR")


def hbs_data():
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    ps = PowerSpecs()
    ps.read_from_txt(HBS)
    return multifidelity_training_set(ps)


def hbs_protocol(X, Y, Xt):
    """tests/test_ho2021_multibin.py:20-43: a fresh MultiFidelityGPModel, optimize(max_iters=100,
    use_adam=True, learning_rate=0.1, unfix_noise_after=50), then predict_f on the test inputs."""
    m = make_model(X, Y)
    m.optimize(max_iters=100, learning_rate=0.1, use_adam=True, unfix_noise_after=50, verbose=False)
    mean, var = m.predict_f(Xt)
    torch.cuda.synchronize()
    return m


def hbs_cold_child():
    """--hbs-cold (run as a child process by hbs_leg): the reference test's protocol ONCE in a
    fresh process, as the reference's test runs it -- kernel code loading, workspace sizing and the
    step-graph capture included (the interpreter start, `import torch` and the CUDA context are
    not: the reference's figure would not include TF's import either)."""
    X, Y, Xt, _ = hbs_data()
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")   # the context
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hbs_protocol(X, Y, Xt)
    dt = time.perf_counter() - t0
    print(json.dumps({"train_predict_s_cold": dt}))
    return 0


def hbs_cold_run():
    """train_predict_s_cold from a child process (None if it fails)."""
    import subprocess
    try:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--hbs-cold"], capture_output=True,
                           text=True, timeout=300)
        for ln in r.stdout.splitlines()[::-1]:
            if ln.startswith("{"):
                return json.loads(ln)["train_predict_s_cold"]
    except (OSError, ValueError, KeyError, subprocess.SubprocessError):
        pass
    return None


def hbs_leg(steps=200, warmup=20):
    """BASELINE configs[1] (Ho-Bird-Shelton 50LF/3HF, D=5, P=49, fp64): pure latency, so the
    figure is wall-clock.
      train_predict_s_cold  the reference's test protocol (hbs_protocol) run ONCE in a fresh child
                            process, capture and kernel loading included (the reference's test runs
                            it once per process);
      train_predict_s       the same protocol in this process after one untimed run: a fresh model
                            then reuses the pooled session's buffers and captured step graphs
                            (models.py session pool), i.e. a warm-pool figure;
      ms_per_step           replayed Adam steps of a session, like the Goku line.
    roofline: at this size (n, p <= 64, D <= 16) the whole value + gradient + Adam step is ONE
    launch of k_gpr_tiny (mfgp_set_tiny, the default), booked under its name with the SURVEY §8(d)
    value+grad flops of the step; latency-bound."""
    X, Y, Xt, _ = hbs_data()
    n, d, P = X.shape[0], X.shape[1] - 1, Y.shape[1]
    cold = hbs_cold_run()
    protocol = lambda: hbs_protocol(X, Y, Xt)
    protocol()
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        protocol()
        ts.append(time.perf_counter() - t0)
    model = make_model(X, Y)
    sess = model.adam_session(0.1, steps + warmup, graph=True, graph_chunk=50)
    sess.run(warmup)
    sess.prepare(steps)
    sess.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sess.run(steps)
    sess.sync()
    dt = time.perf_counter() - t0
    sess.finish()
    roof = roofline(model, n, P, d, pmc=False)
    roof["bound"] = "latency"
    from multi_fidelity_gpflow_amd.engine import Engine
    eng = Engine.get()
    if eng.mode()[2] and n <= 64 and P <= 64 and d <= 16:
        # the one-launch path: every phase mark but the first brackets k_gpr_tiny (or nothing)
        us = sum(roof["phase_ms"].values()) * 1e3
        fl = step_flops(n, P, d)
        roof.update({"kernel": "k_gpr_tiny (the whole LML value + gradient (+ Adam) step in one workgroup)",
                     "launches_per_step": 1, "avg_launch_us": round(us, 3), "flop_per_launch": fl,
                     "achieved": round(fl / (us * 1e-6) / 1e12, 6),
                     "frac": round(fl / (us * 1e-6) / 1e12 / FP64_PEAK_TFLOPS, 8),
                     "flop_source": "SURVEY §8(d) value+grad unit (step_flops)"})
        # the live figures are the same measurement here (no rocprofv3 average for this kernel)
        roof["achieved_live"], roof["frac_live"] = roof["achieved"], roof["frac"]
    return {
        "config": {"workload": "hbs_multibin_adam_step", "n_lf": int((X[:, -1] == 0).sum()),
                   "n_hf": int((X[:, -1] == 1).sum()), "d": d, "p": P},
        "dtype": "f64",
        "train_predict_s_cold": None if cold is None else round(cold, 5),
        "train_predict_s": round(float(np.median(ts)), 5),
        "train_predict_s_note": "warm pool: a fresh model of a seen shape replays the pooled session's graphs",
        "train_predict_s_runs": [round(t, 5) for t in ts],
        "protocol": "tests/test_ho2021_multibin.py:20-43 (optimize 100 Adam steps, lr 0.1, then predict_f(X_test))",
        "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 4),
        "evals_per_s": round(steps / dt, 2),
        "roofline": roof,
    }


def synth_leg(steps=3, warmup=2):
    """BASELINE configs[4] (synthetic N_L=16384, N_H=2048, D=10, P=512, fp32), 1 GPU: replayed
    value+grad+Adam steps (graphs of 2 steps captured in warm-up), roofline of k32_update."""
    from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
    X, Y, Xt, Yt = synthetic_multifidelity()
    n, d, P = X.shape[0], X.shape[1] - 1, Y.shape[1]
    model = make_model(X, Y, "float32")
    sess = model.adam_session(0.1, steps + warmup, graph=True, graph_chunk=2)
    sess.run(warmup)
    sess.prepare(steps)
    sess.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sess.run(steps)
    sess.sync()
    dt = time.perf_counter() - t0
    sess.finish()
    roof = roofline_f32(model, reps=1)
    out = {
        "config": {"workload": "synth_multibin_adam_step", "n_lf": int((X[:, -1] == 0).sum()),
                   "n_hf": int((X[:, -1] == 1).sum()), "d": d, "p": P},
        "dtype": "f32",
        "steps": steps, "warmup": warmup,
        "ms_per_step": round(dt / steps * 1e3, 3),
        "evals_per_s": round(steps / dt, 3),
        "step_tflops": round(step_flops(n, P, d) * steps / dt / 1e12, 2),
        "roofline": roof,
    }
    del sess, model
    torch.cuda.empty_cache()
    return out


def shared_theta_leg(X, Yr, steps, warmup, device):
    """The shared-theta (reference-parity) mode of an N > 1 run: one multi-bin model, each rank
    its contiguous bin block, one RCCL all-reduce of 1 + G doubles per Adam step
    (distributed.SharedThetaTrainer, linear.py:200-214 trajectory).  value = model steps / s
    (strong scaling: the job's total work per step is fixed)."""
    from multi_fidelity_gpflow_amd.distributed import SharedThetaTrainer
    world = dist.get_world_size()
    model = make_model(X, Yr)
    sess = SharedThetaTrainer(model, 0.1, steps + warmup)
    sess.run(warmup)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    sess.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    sess.finish()
    return {"mode": "shared", "scaling": "strong", "steps": steps, "warmup": warmup,
            "ms_per_step": round(dt / steps * 1e3, 4), "value": round(steps / dt, 3), "unit": "evals/s",
            "parallelism": f"bins{world}-shared-theta",
            "collective": collective_label(sess)}


def collective_label(sess) -> str:
    """How a shared-theta trainer ran its per-step all-reduce."""
    backend = dist.get_backend() if dist.is_available() and dist.is_initialized() else "none"
    how = (f"replayed from hipGraphs of {sess.graph_chunk} steps, the all-reduce captured inside"
           if getattr(sess, "graph_chunk", 0) else "eager launches")
    return f"one {backend} all-reduce of 1 + G doubles per step ({how})"


def dist_device_index() -> int:
    """LOCAL_RANK's GPU.  With fewer visible GPUs than ranks (a rehearsal of the N > 1 path on a
    one-GPU box) ranks share devices round-robin."""
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    return local % ndev if ndev > 0 else local


def init_dist(device):
    """RCCL ("nccl") process group; MFGP_DIST_BACKEND=gloo for a rehearsal with several ranks on
    one GPU (RCCL wants one rank per device)."""
    backend = os.environ.get("MFGP_DIST_BACKEND", "nccl")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=device)
    else:
        dist.init_process_group(backend)


def spawn_ranks(n: int) -> int:
    """python -m torch.distributed.run --nproc-per-node n bench.py <same args>, as a child."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--tile", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-train-predict", action="store_true")
    ap.add_argument("--no-latent", action="store_true",
                    help="--config goku_svgp: time the single-bin model only (the PMC passes of tools/gpu_run.sh profile:goku_svgp)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the hbs / synth / goku_svgp sub-objects of the default (Goku, N=1) line")
    ap.add_argument("--mode", choices=["shard", "shared"], default="shard",
                    help="shard: per-shard-theta bin blocks (no inner-loop collective); shared: one model, "
                         "one all-reduce of 1+G doubles per step (reference-parity mode, SURVEY 8(e))")
    ap.add_argument("--hbs-cold", action="store_true", help=argparse.SUPPRESS)   # hbs_leg's child
    ap.add_argument("--config", choices=["goku", "synth", "goku_svgp"], default="goku",
                    help="goku: the BASELINE metric (fp64); synth: BASELINE configs[4] / SURVEY §8(d) "
                         "(N=18432, P=512, fp32)")
    args = ap.parse_args()
    if args.hbs_cold:
        return hbs_cold_child()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        # not launched by torchrun: start one rank per GPU (before this process touches the GPU)
        sys.exit(spawn_ranks(args.gpus))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}")
    if args.config == "synth":
        args.no_cpu_baseline = True
        args.no_train_predict = True
    if args.config == "goku_svgp":
        return bench_svgp(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > max(torch.cuda.device_count(), 1):
        # ranks share a device (a rehearsal on fewer GPUs): persistent flows of different
        # processes cannot all be resident (the library's fence is per process), so use the
        # launch-per-step Cholesky
        os.environ["MFGP_FLOW"] = "0"
        if rank == 0:
            print("bench.py: more ranks than GPUs, persistent Cholesky disabled (MFGP_FLOW=0)", file=sys.stderr)
    local = dist_device_index()
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    # MFGP_DIST_WS1=1: a process group even at world size 1 (the RCCL code path on one GPU: its
    # broadcast, all-reduce and captured collectives; not a scaling figure)
    ws1 = world == 1 and os.environ.get("MFGP_DIST_WS1", "0") == "1"
    if world > 1 or ws1:
        init_dist(device)

    from multi_fidelity_gpflow_amd.engine import Engine
    eng = Engine.get(device)
    if args.tile:
        eng.set_tile(args.tile)

    if args.config == "synth":
        from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
        X, Y, Xt, Yt = synthetic_multifidelity()   # deterministic: every rank builds the same set
    else:
        X, Y, Xt, Yt = broadcast_inputs(rank, world, device)
    n, d, P = X.shape[0], X.shape[1] - 1, Y.shape[1]
    from multi_fidelity_gpflow_amd.distributed import bin_block
    b0, b1 = bin_block(P, rank, world)
    Yr = np.ascontiguousarray(Y[:, b0:b1])

    synth = args.config == "synth"
    dtype = "float32" if synth else None
    model = make_model(X, Yr, dtype)
    K, W = args.steps, args.warmup
    if args.mode == "shared":
        from multi_fidelity_gpflow_amd.distributed import SharedThetaTrainer
        sess = SharedThetaTrainer(model, 0.1, K + W)
    else:
        sess = model.adam_session(0.1, K + W, graph=True, graph_chunk=50 if args.config == "goku" else 2)
    sess.run(W)
    if hasattr(sess, "prepare"):
        sess.prepare(K)   # capture every graph the timed run replays: the timed region is replay-only
    sess.sync()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    sess.run(K)
    sess.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        dist.barrier()
        t = torch.tensor([dt], dtype=torch.float64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    sess.finish()

    # train + predict wall-clock (notebook protocol, fresh model).  The process's first predict_f
    # loads the predict kernels' code and sizes their workspace (~60 ms once per process,
    # tools/tp_breakdown.py); it runs untimed on the bench model first, like the step warm-up.
    tp = None
    if not args.no_train_predict:
        model.predict_f(Xt)
        torch.cuda.synchronize()
        m2 = make_model(X, Yr, dtype)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        m2.optimize(max_iters=1000, learning_rate=0.1, use_adam=True, unfix_noise_after=500, verbose=False)
        mean, var = m2.predict_f(Xt)
        torch.cuda.synchronize()
        tp = time.perf_counter() - t1
        if world > 1:
            t = torch.tensor([tp], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            tp = float(t.item())

    # N > 1, shard mode: the reference-parity figure of the same job beside it -- ONE model trained
    # with the reference's trajectory (SharedThetaTrainer: every rank its bin block, one all-reduce
    # of 1 + G doubles per step), so a scaling run records both
    shared_sub = None
    if world > 1 and args.mode == "shard" and not synth:
        shared_sub = shared_theta_leg(X, Yr, min(K, 100), min(W, 10), device)

    roof = roofline_f32(model) if synth else roofline(model, n, Yr.shape[1], d)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(X, Y)

    if rank == 0:
        shared = args.mode == "shared"
        value = (K if shared else world * K) / dt
        line = {
            "metric": ("LML evals/sec (synthetic 16384LF/2048HF D=10 P=512, value+grad+Adam step)" if synth else
                       "LML evals/sec (Goku 1128LF/36HF multi-bin, value+grad+Adam step)"),
            "value": round(value, 3),
            "unit": "evals/s",
            "n_gpus": world,
            "steps": K,
            "warmup": W,
            "ms_per_step": round(dt / K * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if shared else "weak",
            "vs_baseline": None,
            "dtype": "f32" if synth else "f64",
            "data": ("synthetic (SURVEY §8(d) recipe, seed 20251015), built on every rank" if synth else
                     "Goku z=0 P(k) (reference data files, tests/golden/data), " + bcast_label(world)),
            "config": {"workload": "synth_multibin_adam_step" if synth else "goku_multibin_adam_step",
                       "n_lf": int((X[:, -1] == 0).sum()), "n_hf": int((X[:, -1] == 1).sum()), "d": d, "p": P,
                       "bins_per_rank": Yr.shape[1], "tile": eng.tile(),
                       "parallelism": (f"bins{world}-shared-theta" if shared else f"bins{world}") if world > 1
                       else "single", "mode": args.mode},
            "bin_throughput": round(P * K / dt, 2),
            "train_predict_s": None if tp is None else round(tp, 4),
            "step_tflops": round(step_flops(n, P, d) * value / 1e12, 4),
            "roofline": roof,
            "cpu_baseline": cpu,
            "published_m1_cpu": None if synth else {"train_1000_adam_s": 142.36, "evals_per_s": 7.02,
                                                    "source": "notebooks/demo: goku power spectra.ipynb:120"},
        }
        if shared_sub is not None:
            line["shared_theta"] = shared_sub
        if args.mode == "shared":
            line["collective"] = collective_label(sess)
        if world == 1 and args.config == "goku" and not args.no_extras:
            # every other BASELINE config, measured in this process after the headline timing
            line["hbs"] = hbs_leg()
            line["goku_svgp"] = svgp_leg(X, Yr, Xt, 20, 5)
            line["synth"] = synth_leg()
        print(json.dumps(line))
    if world > 1 or ws1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
