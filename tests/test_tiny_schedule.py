"""k_gpr_tiny's LDS slots and barriers, restated on the CPU.

The one-workgroup small-problem kernel (csrc/mfgp_kernels.hip k_gpr_tiny) keeps every operand in
16 LDS tile slots that are reused across its stages, with only workgroup barriers to order one
wave's LDS accesses against another's.  This test restates, element by element, which LDS doubles
every wave reads and writes between consecutive barriers, for every shape the kernel handles
(T, Tp, Ts in {1, 2}; value only / value + gradient; predict_f), and checks:

  * no hazard: two accesses to the same LDS double by DIFFERENT waves with at least one write are
    never in the same barrier interval (within one wave, LDS accesses are in program order);
  * every barrier is needed: merging the two intervals on either side of barrier k produces a hazard
    in at least one configuration;
  * the restatement is the kernel's schedule: the barriers of k_gpr_tiny's body, in source order,
    are exactly TINY_BARRIER(1) .. TINY_BARRIER(19) and the body has no other workgroup barrier.
So deleting any one barrier from the kernel fails the third check, and the second says why it was
there.  Index arithmetic below follows the kernel's (TileCfg<32>: stride S = 34, E = 1088 doubles a
slot; Acc<32>: wave w owns output block (w >> 1, w & 1) of 16 x 16; tile_mma reads op(A)'s row block
and op(B)'s column block of its output block, all 32 k)."""
import itertools
import os
import re

import numpy as np

from conftest import ROOT

S, E, NT = 34, 34 * 32, 256
XS, TN, MAXD = 17, 64, 16
NBAR = 19


def slot(i):
    return i * E


# slot 12 (misc): dg | bad | il | il2 | red | gsh | tsh | lv (double-cell offsets)
MISC = slot(12)
DG, BAD, IL = MISC, MISC + 64, MISC + 66
IL2 = IL + 2 * MAXD
RED = IL2 + 2 * MAXD
GSH = RED + 4 * (2 * MAXD + 6)
TSH = GSH + 2 * MAXD + 6            # int array: two ints a cell
LV = GSH + 2 * (2 * MAXD + 6)
XR = slot(11)
AL, AD = slot(6), slot(6) + TN * XS
NL = AD + TN * XS
ND, FL = NL + TN, NL + 2 * TN
K00, K10, K11, D0, D1, L10 = (slot(i) for i in range(6))


def Yt(r, c):
    return slot(6 + 2 * r + c)


def ELt(tl):
    return slot(13 + tl)


def wave_of(t):
    return t // 64


class Sched:
    def __init__(self):
        self.epoch = 0
        self.bars = []          # barrier label of each epoch boundary, in execution order
        self.ev = []            # (epoch, wave, is_write, cells ndarray)

    def bar(self, k):
        self.bars.append(k)
        self.epoch += 1

    def acc(self, w, write, cells):
        cells = np.unique(np.asarray(list(cells), dtype=np.int64))
        if cells.size:
            self.ev.append((self.epoch, w, write, cells))

    def rd(self, w, cells):
        self.acc(w, False, cells)

    def wr(self, w, cells):
        self.acc(w, True, cells)

    # ---- access patterns of the kernel's helpers
    def strided(self, count, cell, write, cond=lambda e: True):
        """for (e = t; e < count; e += 256): element e by thread e % 256"""
        per = {w: [] for w in range(4)}
        for e in range(count):
            if cond(e):
                c = cell(e)
                for x in (c if isinstance(c, (list, tuple)) else [c]):
                    per[wave_of(e % NT)].append(x)
        for w, cs in per.items():
            self.acc(w, write, cs)

    def mma(self, A, ta, B, tb):
        """tile_mma<32, ta, tb>(acc, A, B): wave w reads op(A) rows rb.., op(B) cols cb.. (all k)"""
        for w in range(4):
            rb, cb = 16 * (w >> 1), 16 * (w & 1)
            ks = range(32)
            a = [A + k * S + i if ta else A + i * S + k for i in range(rb, rb + 16) for k in ks]
            b = [B + j * S + k if tb else B + k * S + j for j in range(cb, cb + 16) for k in ks]
            self.rd(w, a + b)

    def own(self, X, write):
        """acc_to_lds / acc_load: wave w's own 16 x 16 block"""
        for w in range(4):
            rb, cb = 16 * (w >> 1), 16 * (w & 1)
            self.acc(w, write, [X + (rb + i) * S + cb + j for i in range(16) for j in range(16)])

    def factor(self, X, R, dgo, bad):
        """tile_potrf_inv_w1_wave(X, S, X, R, dg + dgo, bad): wave 0 alone"""
        tile = [X + i * S + j for i in range(32) for j in range(32)]
        self.rd(0, tile)
        self.wr(0, tile)
        self.wr(0, [R + i * S + j for i in range(32) for j in range(32)])
        self.wr(0, [DG + dgo + i for i in range(32)] + [bad])


def tiny_schedule(n, p, D, want_grad, pred=False, ns=0):
    """Execution of k_gpr_tiny<pred> (csrc/mfgp_kernels.hip) on an (n, p, D) problem, as LDS
    accesses per wave between barriers (interval i lies between the i-th and (i+1)-th barrier)."""
    T, Tp = (n + 31) // 32, (p + 31) // 32
    G = 2 * D + 4
    D4 = (D + 3) & ~3
    s = Sched()

    def bar(k):
        s.bar(k)

    # stage: raw rows, lengthscale reciprocals
    s.strided(TN * XS, lambda e: XR + e, True)
    for t in range(D):
        s.wr(wave_of(t), [IL + t, IL + MAXD + t, IL2 + t, IL2 + MAXD + t, LV + t, LV + MAXD + t])
    bar(1)
    s.strided(TN * XS, lambda e: XR + e, False)
    s.strided(TN * XS, lambda e: [IL + e % XS, IL + MAXD + e % XS] if e % XS < D else [], False)
    s.strided(TN * XS, lambda e: [AL + e, AD + e], True)
    for t in range(TN):
        s.rd(wave_of(t), [XR + t * XS + D] if t < n else [])
        s.wr(wave_of(t), [FL + t])
    bar(2)
    for t in range(TN):
        s.rd(wave_of(t), [AL + t * XS + d for d in range(D4)] + [AD + t * XS + d for d in range(D4)])
        s.wr(wave_of(t), [NL + t, ND + t])
    bar(3)
    # Gram: wave w forms blocks 3w .. 3w + 2 of the three lower tiles
    for w in range(4):
        for bq in range(3):
            blk = 3 * w + bq
            tl, sub = blk >> 2, blk & 3
            ti, tj = (0 if tl == 0 else 1), (1 if tl == 2 else 0)
            if ti >= T:
                continue
            rb, cb = 2 * ti + (sub >> 1), 2 * tj + (sub & 1)
            rows = [16 * rb + i for i in range(16)] + [16 * cb + i for i in range(16)]
            s.rd(w, [A + r * XS + d for A in (AL, AD) for r in rows for d in range(D4)])
            s.rd(w, [X + r for X in (NL, ND, FL) for r in rows])
            out = [(16 * rb + i - 32 * ti) * S + 16 * cb + j - 32 * tj for i in range(16) for j in range(16)]
            s.wr(w, [ELt(tl) + o for o in out] + [slot(tl) + o for o in out])
    bar(4)
    s.factor(K00, D0, 0, BAD)
    bar(5)
    if T > 1:
        s.mma(K10, False, D0, True)
        s.own(L10, True)
        bar(6)
        s.own(K11, False)
        s.mma(L10, False, L10, True)
        s.own(K11, True)
        s.mma(L10, False, D0, False)
        s.own(K10, True)
        bar(7)
        s.factor(K11, D1, 32, BAD)
        bar(8)
        s.mma(D1, False, K10, False)
        s.own(L10, True)
    s.strided(T * Tp * 1024, lambda e: Yt((e >> 10) // Tp, (e >> 10) % Tp) + ((e >> 5) & 31) * S + (e & 31), True)
    bar(9)
    for c in range(Tp):
        s.mma(D0, False, Yt(0, c), False)
        if T > 1:
            s.mma(L10, False, Yt(0, c), False)
            s.mma(D1, False, Yt(1, c), False)
    if not pred:
        s.mma(D0, True, D0, False)
        if T > 1:
            s.mma(L10, True, L10, False)
        s.own(K00, True)
        if T > 1:
            s.mma(D1, True, L10, False)
            s.own(K10, True)
            s.mma(D1, True, D1, False)
            s.own(K11, True)
    bar(10)
    for c in range(Tp):
        s.own(Yt(0, c), True)
        if T > 1:
            s.own(Yt(1, c), True)
    bar(11)
    if pred:
        Ts = (ns + 31) // 32
        XSS = slot(13)

        def Km(i, c):
            return slot(c if i == 0 else (2 if c == 0 else 10))
        s.strided(TN * XS, lambda e: XSS + e, True)
        bar(12)

        def km_cells(e):
            tl, r, c = e >> 10, (e >> 5) & 31, e & 31
            ti, tc = tl // Ts, tl % Ts
            gi, gs = 32 * ti + r, 32 * tc + c
            return gi, gs, Km(ti, tc) + r * S + c
        per_r = {w: [] for w in range(4)}
        for e in range(T * Ts * 1024):
            gi, gs, cell = km_cells(e)
            w = wave_of(e % NT)
            s.wr(w, [cell])
            if gi < n and gs < ns:
                per_r[w] += [XR + gi * XS + d for d in range(D + 1)] + [XSS + gs * XS + d for d in range(D + 1)]
                per_r[w] += [IL2 + d for d in range(D)] + [IL2 + MAXD + d for d in range(D)]
        for w, cs in per_r.items():
            s.rd(w, cs)
        bar(13)
        for c in range(Ts):
            s.mma(D0, False, Km(0, c), False)
            if T > 1:
                s.mma(L10, False, Km(0, c), False)
                s.mma(D1, False, Km(1, c), False)
        bar(14)
        for c in range(Ts):
            s.own(Km(0, c), True)
            if T > 1:
                s.own(Km(1, c), True)
        bar(15)
        for cs in range(Ts):
            for cy in range(Tp):
                s.mma(Km(0, cs), True, Yt(0, cy), False)
                if T > 1:
                    s.mma(Km(1, cs), True, Yt(1, cy), False)
        for t in range(ns):
            cs, cc = t >> 5, t & 31
            s.rd(wave_of(t), [Km(i, cs) + r * S + cc for i in range(T) for r in range(32)] + [XSS + t * XS + D])
        s.rd(0, [BAD])
        return s
    for c in range(Tp):
        s.mma(D0, True, Yt(0, c), False)
        if T > 1:
            s.mma(L10, True, Yt(1, c), False)
            s.mma(D1, True, Yt(1, c), False)
    bar(16)
    for c in range(Tp):
        s.own(Yt(0, c), True)
        if T > 1:
            s.own(Yt(1, c), True)
    for t in range(min(n, TN)):
        s.rd(wave_of(t), [DG + t])
    bar(17)
    if want_grad:
        for tl in range(3):
            if tl > 0 and T < 2:
                continue
            ti, tj = (0 if tl == 0 else 1), (1 if tl == 2 else 0)
            s.own(slot(tl), False)
            for c in range(Tp):
                s.mma(Yt(ti, c), False, Yt(tj, c), True)
            s.own(ELt(tl), False)
            for w in range(4):
                rb, cb = 16 * (w >> 1), 16 * (w & 1)
                rows = [32 * ti + rb + i for i in range(16)] + [32 * tj + cb + j for j in range(16)]
                s.rd(w, [XR + r * XS + d for r in rows if r < n for d in range(D + 1)])
                s.rd(w, [IL2 + MAXD + d for d in range(D)])
    # reduction partials: RB = slot 3 onwards, quantity q's 64 partials, wave w's 16 of them
    RB = slot(3)
    qs = list(range(G + 2)) if want_grad else [G, G + 1]
    for w in range(4):
        s.wr(w, [RB + q * 64 + 16 * w + i for q in qs for i in range(16)])
    bar(18)
    for g0 in range(0, G + 2, NT // 8):
        for t in range(NT):
            qx, sub = g0 + (t >> 3), t & 7
            if qx < G + 2 and (want_grad or qx >= G):
                s.rd(wave_of(t), [RB + qx * 64 + sub * 8 + u for u in range(8)])
            if sub == 0 and qx < G + 2:
                if 1 <= qx <= D:
                    s.rd(wave_of(t), [LV + qx - 1])
                elif 2 + D <= qx <= 1 + 2 * D:
                    s.rd(wave_of(t), [LV + MAXD + qx - 2 - D])
                s.wr(wave_of(t), [GSH + (2 + qx if qx < G else qx - G)])
    for aq in range(G):   # wave 1's Adam owners: tsh[aq] (two ints a cell)
        s.wr(wave_of(64 + aq), [TSH + aq // 2])
    s.rd(0, [BAD])
    bar(19)
    for t in range(NT):
        s.rd(wave_of(t), [BAD, GSH, GSH + 1])
    for aq in range(G):
        s.rd(wave_of(64 + aq), [GSH + 2 + aq] + [TSH + r // 2 for r in range(G)])
    if want_grad:
        for q in range(G):
            s.rd(wave_of(q), [GSH + 2 + q])
    return s


def _conflict(evs):
    """First LDS double that two different waves touch in `evs` (one interval) with at least one
    write, or None: per cell the mask of waves accessing it and of waves writing it."""
    if not evs:
        return None
    cells = np.concatenate([c for _, _, c in evs])
    acc = np.concatenate([np.full(c.size, 1 << w, np.int64) for w, _, c in evs])
    wrt = np.concatenate([np.full(c.size, (1 << w) if wr else 0, np.int64) for w, wr, c in evs])
    order = np.argsort(cells, kind="stable")
    cells, acc, wrt = cells[order], acc[order], wrt[order]
    starts = np.flatnonzero(np.r_[True, cells[1:] != cells[:-1]])
    am = np.bitwise_or.reduceat(acc, starts)
    wm = np.bitwise_or.reduceat(wrt, starts)
    multi_writer = (wm & (wm - 1)) != 0
    bad = (wm != 0) & (multi_writer | ((am & ~wm) != 0))
    return int(cells[starts[np.argmax(bad)]]) if bad.any() else None


def _epochs(s):
    by = {}
    for ep, w, wr, cells in s.ev:
        by.setdefault(ep, []).append((w, wr, cells))
    return by


def hazards(s):
    """Cross-wave conflicts inside one barrier interval: [(interval, first cell)]."""
    out = []
    for ep, evs in sorted(_epochs(s).items()):
        c = _conflict(evs)
        if c is not None:
            out.append((ep, c))
    return out


def hazard_without(s, i):
    """The conflict that appears when the i-th executed barrier of `s` is removed (its two
    intervals merge), or None."""
    by = _epochs(s)
    return _conflict(by.get(i, []) + by.get(i + 1, []))


CONFIGS = [dict(n=n, p=p, D=D, want_grad=g) for n in (20, 53) for p in (20, 49) for D in (1, 5) for g in (0, 1)] + \
          [dict(n=n, p=p, D=3, want_grad=0, pred=True, ns=ns) for n in (20, 53) for p in (20, 49) for ns in (9, 40)]


def test_tiny_schedule_has_no_cross_wave_hazard():
    for cfg in CONFIGS:
        s = tiny_schedule(**cfg)
        assert not hazards(s), (cfg, hazards(s)[:3])


def test_every_tiny_barrier_is_needed():
    needed = set()
    for cfg in CONFIGS:
        s = tiny_schedule(**cfg)
        for i, k in enumerate(s.bars):
            if hazard_without(s, i) is not None:
                needed.add(k)
    assert needed == set(range(1, NBAR + 1)), f"barriers ordering nothing: {sorted(set(range(1, NBAR + 1)) - needed)}"


def _tiny_body():
    src = open(os.path.join(ROOT, "multi_fidelity_gpflow_amd", "csrc", "mfgp_kernels.hip")).read()
    i = src.index("void k_gpr_tiny(TinyArgs a) {")
    j, depth = src.index("{", i), 0
    for k in range(j, len(src)):
        depth += {"{": 1, "}": -1}.get(src[k], 0)
        if depth == 0:
            return src[j:k + 1]
    raise AssertionError("k_gpr_tiny body not found")


def test_kernel_barriers_are_the_restated_ones():
    body = re.sub(r"//[^\n]*", "", _tiny_body())
    assert "__syncthreads" not in body, "k_gpr_tiny: a workgroup barrier outside TINY_BARRIER(k)"
    labels = [int(x) for x in re.findall(r"TINY_BARRIER\((\d+)\)", body)]
    assert labels == list(range(1, NBAR + 1)), labels
    # every restated barrier executes in some configuration, in the source order
    seen = set()
    for cfg in CONFIGS:
        bars = tiny_schedule(**cfg).bars
        assert bars == sorted(bars), (cfg, bars)
        seen |= set(bars)
    assert seen == set(range(1, NBAR + 1))
