"""Timeline of the persistent dataflow Cholesky (k_chol_flow) at Goku: the diag chain per step
and the worker waves' busy / waiting split.  Diagnostic only (GPU box):
    python tools/flow_trace.py [reps]"""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from multi_fidelity_gpflow_amd import _lib                       # noqa: E402
from multi_fidelity_gpflow_amd.engine import Engine             # noqa: E402
from oracle import mfgp_oracle as O                             # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    d = O.load_powerspecs(os.path.join(ROOT, "tests", "golden", "data",
                                       "matter_power_1128_Box1000_Part750_36_Box1000_Part3000_z0"))
    X, Y = d["X"], d["Y"]
    eng = Engine.get()
    lib = eng.lib
    _lib.check(lib.mfgp_set_flow(eng.h, 2), "mfgp_set_flow")
    n, p, D = X.shape[0], Y.shape[1], X.shape[1] - 1
    Xd = torch.tensor(X, device=eng.device)
    Yd = torch.tensor(Y, device=eng.device)
    th = torch.tensor(np.concatenate([[1.0], np.ones(D), [1.0], np.ones(D), [1.0, 1e-3]]), device=eng.device)
    off, cnt = C.c_size_t(), C.c_int()
    _lib.check(lib.mfgp_gpr_flow_trace(eng.h, n, p, D, C.byref(off), C.byref(cnt)), "trace")
    T = (n + 31) // 32
    for r in range(reps):
        out, info = eng.gpr_lml(Xd, Yd, th, want_grad=True)
        torch.cuda.synchronize()
    ws = eng._ws["gpr"]
    tr = ws[off.value: off.value + 8 * cnt.value].view(torch.int64).cpu().numpy() / 100.0   # us
    st, rdy, fs, pub = tr[:T], tr[T:2 * T], tr[2 * T:3 * T], tr[3 * T:4 * T]
    print(f"info {int(info.item())}  lml {float(out[0]):.6f}")
    print(f"gram phase (us from launch): wave 0's block of (0,0) {st[0]:.2f}, waves 1 / 4's {rdy[0]:.2f},"
          f" wave 2's A(1,0) {fs[0]:.2f}")
    r2, pp, qq, l2 = tr[4 * T:5 * T], tr[5 * T:6 * T], tr[6 * T:7 * T], tr[7 * T:8 * T]
    print(" k   start  A'ready  wait  factor  publish  step | got A(k,k-2) A(k,k-1) A(k,k)  L(k,k-2)  (rel. to publish of D_k-3)")
    for k in range(1, T):
        ref = pub[k - 3] if k >= 3 else 0.0
        print(f"{k:2d} {st[k]:7.2f} {rdy[k]:7.2f} {rdy[k]-st[k]:5.2f} {fs[k]:7.2f} {pub[k]:7.2f} {pub[k]-pub[k-1]:5.2f}"
              f" | {r2[k]-ref:6.2f} {pp[k]-ref:6.2f} {qq[k]-ref:6.2f} {l2[k]-ref:6.2f}")
    Wn = (cnt.value - 8 * T - 6 * T - 5 * (T * (T + 1) // 2 + 4)) // (3 + 4 * 40)
    w = tr[8 * T: 8 * T + 3 * Wn].reshape(-1, 3)
    busy = w[:, 1] > 0
    w = w[busy]
    print(f"workers with items: {len(w)}  done: max {w[:,1].max():.1f} us  median {np.median(w[:,1]):.1f}"
          f"  first-item start median {np.median(w[:,0]):.2f}  waiting: mean {w[:,2].mean():.1f} us"
          f" max {w[:,2].max():.1f}")
    late = np.argsort(-w[:, 1])[:8]
    print("latest workers (start, done, waited):", [tuple(np.round(w[i], 1)) for i in late])
    W = (cnt.value - 8 * T - 6 * T - 5 * (T * (T + 1) // 2 + 4)) // (3 + 4 * 40)
    w5 = tr[8 * T + 3 * W + 4 * 40 * W: 8 * T + 3 * W + 4 * 40 * W + 6 * T]
    print(" j  got A(j,j-2) | gate open  waits done  L(j,j-2)   (wave 5, us after D_j-3 published; D_j-2 at)")
    for j in range(4, T):
        ref = pub[j - 3]
        print(f"{j:2d} {r2[j]-ref:6.2f} | {w5[j]-ref:6.2f} {w5[T + j]-ref:6.2f} {l2[j]-ref:6.2f}   D_j-2 {pub[j-2]-ref:5.2f}"
              f"  P2(j-1)~{fs[j-1]-ref:5.2f}")
    print(" k  | chain: start  A'ready  fstart | w5 L(k,k-2) | w6 waits  done | w7 waits  done   (us after D_k-2 factor start)")
    for k in range(4, T):
        ref = fs[k - 2]
        print(f"{k:2d}  | {st[k]-ref:6.2f} {rdy[k]-ref:7.2f} {fs[k]-ref:7.2f} | {l2[k]-ref:9.2f} |"
              f" {w5[2 * T + k]-ref:7.2f} {w5[3 * T + k]-ref:6.2f} | {w5[4 * T + k]-ref:7.2f} {w5[5 * T + k]-ref:6.2f}")
    G = T * (T + 1) // 2 + 4   # k_gram timeline: [3 G] stamps, then [2 G] (mfgp_flow.h flow_gram_dbg_count)
    g = ws[off.value + 8 * (cnt.value - 5 * G): off.value + 8 * cnt.value].view(torch.int64).cpu().numpy()[:3 * G].reshape(-1, 3)
    gg = g.astype(np.float64) / 100.0
    ext = [(i, gg[i, 2]) for i in range(len(gg)) if gg[i, 0] == 0 and gg[i, 2] > 0]
    print("k_gram extra workgroups (index, us to done):", [(i, round(v, 2)) for i, v in ext])
    print("k_gram WG 0 (staged, entries, done):", gg[0], " latest:",
          [(int(i), gg[i, 2]) for i in np.argsort(-gg[:, 2])[:6]])
    g = g[g[:, 2] > 0].astype(np.float64) / 100.0
    if len(g):
        print(f"k_gram per workgroup (us since its start): staged median {np.median(g[:, 0]):.2f} max {g[:, 0].max():.2f};"
              f" entries done median {np.median(g[:, 1]):.2f} max {g[:, 1].max():.2f}; end median {np.median(g[:, 2]):.2f}"
              f" max {g[:, 2].max():.2f}")
    its = items(tr, T, W)
    names = {0: "A", 1: "R", 2: "al", 3: "H"}
    for kk in (12, 20, 28):
        print(f"-- items feeding chain step {kk} (D_{kk-3} published at {pub[kk-3]:.2f}):")
        want = {(0, kk, kk - 1), (0, kk, kk - 2), (0, kk, kk), (0, kk, kk - 4), (0, kk - 1, kk - 4),
                (0, kk, kk - 3), (0, kk - 1, kk - 5), (0, kk, kk - 5)}
        print(f"   (D_{kk-5} {pub[kk-5]:.2f}  D_{kk-4} {pub[kk-4]:.2f}  D_{kk-3} {pub[kk-3]:.2f})")
        for (wv, code, lev, b, r, e) in its:
            ty, i, j = (code >> 20) & 15, (code >> 10) & 1023, code & 1023
            if (ty, i, j) in want and lev >= kk - 7:
                print(f"   {names[ty]}({i},{j}) lvl {lev:2d}: begin {b:7.2f} ready {r:7.2f} end {e:7.2f}  (work {e-r:5.2f})")
    # lag of the L^{-1} / Z / alpha pipelines behind the chain: per level, latest item end - D_l published
    print(" lvl  D_l    A-fin lag  R-fin lag  Y-fin lag  alpha lag   (us after D_l published)")
    for lev in range(0, T, 3):
        row = []
        for kind in ("A", "R", "Y", "al"):
            ends = []
            for (wv, code, lv, b, r, e) in its:
                ty, i, j = (code >> 20) & 15, (code >> 10) & 1023, code & 1023
                k2 = {0: "A", 1: ("Y" if j >= T else "R"), 2: "al", 3: "H"}[ty]
                if k2 != kind:
                    continue
                # the item that completes level lev: finalize at lev (merged: update at lev-1) / alpha update at lev
                if (kind == "A" and lv == lev - 1 and j == lev) or (kind in ("R", "Y") and lv == lev and i == lev) or \
                   (kind == "al" and lv == lev):
                    ends.append(e)
            row.append(max(ends) - pub[lev] if ends else float("nan"))
        print(f" {lev:3d} {pub[lev]:7.2f} " + " ".join(f"{v:9.2f}" for v in row))
    Tm = T - 1
    print(f"-- tail: last items of row {Tm} R / Y tiles and alpha tiles (D_{Tm} published at {pub[Tm]:.2f})")
    for (wv, code, lv, b, r, e) in sorted(its, key=lambda x: x[5]):
        ty, i, j = (code >> 20) & 15, (code >> 10) & 1023, code & 1023
        if lv < Tm - 3:
            continue
        if (ty == 1 and i == Tm and (j in (0, 10, 20, 30, Tm - 1) or j >= T)) or (ty == 2 and i in (0, 20, Tm)):
            print(f"   {names[ty]}({i},{j}) lvl {lv:2d}: begin {b:7.2f} ready {r:7.2f} end {e:7.2f}  (work {e-r:5.2f})")
    dur = np.array([e - r for (_, _, _, b, r, e) in its])
    print(f"item work time (after waits): median {np.median(dur):.2f} us  p90 {np.percentile(dur, 90):.2f}  max {dur.max():.2f}")


def items(tr, T, W, LOG=40):
    """Per-item log: rows (wave, code, level, begin, ready, end) in us."""
    e = tr[8 * T + 3 * W: 8 * T + 3 * W + W * LOG * 4].reshape(W, LOG, 4)
    out = []
    for w in range(W):
        for n in range(LOG):
            c = int(round(e[w, n, 0] * 100.0))
            if e[w, n, 3] <= 0:
                continue
            out.append((w, c >> 8, c & 255, e[w, n, 1], e[w, n, 2], e[w, n, 3]))
    return out


if __name__ == "__main__":
    main()
