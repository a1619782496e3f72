#!/usr/bin/env python
"""SVGP training step timing on Goku (README.md:86-87 configurations):
single-bin SVGP (M=300, one latent per bin, P=64) and latent SVGP (L=15, M=300).
Prints one JSON line per model: seconds per optimize() iteration (hipGraph replay)."""
import argparse, json, os, sys, time
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import multi_fidelity_gpflow_amd as M
from bench import load_goku

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--which", default="both")
a = ap.parse_args()
X, Y, Xt, Yt = load_goku()
D, P = X.shape[1] - 1, Y.shape[1]
k = lambda: M.SquaredExponential(lengthscales=np.ones(D))
res = []
if a.which in ("both", "single"):
    m = M.SingleBinSVGP(X, Y, k(), k(), P, Z=np.zeros((300, D + 1)))
    tr = M.svgp._SVGPTrainer(m, (X, Y), max_iters=a.iters + 10, initial_lr=0.1, graph=True, graph_chunk=10)
    tr.run(10); tr.sync()
    t0 = time.perf_counter(); tr.run(a.iters); tr.sync(); dt = (time.perf_counter() - t0) / a.iters
    res.append({"model": "SingleBinSVGP goku M=300 L=P=64", "s_per_iter": dt,
                "ref_m1_s_per_iter": 2237.47 / 1000, "loss_last": tr.loss_at(a.iters + 9)})
if a.which in ("both", "latent"):
    m = M.LatentMFCoregionalizationSVGP(X, Y, k(), k(), num_latents=15, num_inducing=300, num_outputs=P)
    tr = M.svgp._SVGPTrainer(m, (X, Y), max_iters=a.iters + 10, initial_lr=0.1, graph=True, graph_chunk=10)
    tr.run(10); tr.sync()
    t0 = time.perf_counter(); tr.run(a.iters); tr.sync(); dt = (time.perf_counter() - t0) / a.iters
    res.append({"model": "LatentMFCoregionalizationSVGP goku L=15 M=300", "s_per_iter": dt,
                "ref_m1_s_per_iter": 1020.22 / 2000, "loss_last": tr.loss_at(a.iters + 9)})
for r in res:
    print(json.dumps(r))
