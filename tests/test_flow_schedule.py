"""Host-side check of the k_chol_flow schedule (csrc/mfgp_flow.h, csrc/mfgp_flow.hip), no GPU.

The persistent Cholesky launch is correct only if (1) the owner table hands every output tile to
exactly one worker wave and (2) the waves' level-ordered item programs, together with the diag
workgroup's chain, can always run to completion (every wait is eventually satisfied: no cycle).
This restates the device's tile catalogue (flow_nA / flow_decode / flow_tile / build_flow_owner)
and each item's inputs, and runs the programs as a dependency simulation for Goku's T = 37 and
for small / ragged tile counts and small wave counts (several tiles per wave, where the order of
items inside a wave matters)."""
import pytest

FT_A, FT_R, FT_AL, FT_G = 0, 1, 2, 4
G_TILES = [(3, 1), (3, 2), (3, 3)]   # flow_gtile (rows 0-2: the diag workgroup's Gram phase)
MAXOWN = 4


def tri(t):
    i = 0
    while (i + 1) * (i + 2) // 2 <= t:
        i += 1
    return i, t - i * (i + 1) // 2


def n_a(T):
    return T * (T + 1) // 2 - 9 if T >= 4 else 0


def n_g(T):
    return sum(1 for i, _ in G_TILES if i < T)


def ntiles(T, Tp):
    return n_a(T) + T * (T - 1) // 2 + 2 * T * Tp + n_g(T)


def decode(g, T, Tp):
    nA = n_a(T)
    if g < nA:
        return (FT_A,) + tri(6 if g == 0 else g + 9)
    g -= nA
    nR = T * (T - 1) // 2
    if g < nR:
        i, j = tri(g)
        return (FT_R, i + 1, j)
    g -= nR
    if g < T * Tp:
        return (FT_R, g // Tp, T + g % Tp)
    g -= T * Tp
    if g < T * Tp:
        return (FT_AL, g // Tp, g % Tp)
    g -= T * Tp
    return (FT_G,) + G_TILES[g]


def tile(code, T):
    """(lo, hi, fin, pub) as flow_tile()."""
    ty, i, j = code
    if ty == FT_A:
        if i <= j + 2:
            return 0, i - 4, -1, True
        return 0, j - 1, j, False
    if ty == FT_R:
        return (j if j < T else 0), i - 1, i, False      # every panel, the finalize merged into the last
    if ty == FT_AL:
        return i, T - 1, -1, False
    return 0, -1, -1, False                             # FT_G: formed in the Gram phase, no items


def items(code, T):
    lo, hi, fin, _ = tile(code, T)
    return (hi - lo + 1 if hi >= lo else 0) + (1 if fin >= 0 else 0)


def owner_table(T, Tp, W):
    """build_flow_owner: tiles by descending item count, snake-dealt over W waves (stable order
    here; on the device the order inside one item count is arbitrary, which the simulation below
    covers by also trying the reversed order)."""
    codes = [decode(g, T, Tp) for g in range(ntiles(T, Tp))]
    codes.sort(key=lambda c: -items(c, T))
    own = [[None] * MAXOWN for _ in range(W)]
    for p, c in enumerate(codes):
        r, q = divmod(p, W)
        sn = W - 1 - q if r & 1 else q
        # snake position -> wave: wave 0 of every workgroup first, then wave 1, ... (8 waves per
        # workgroup; waves w and w + 4 share a SIMD)
        nwg = W // 8
        w = (sn % nwg) * 8 + sn // nwg if W % 8 == 0 else sn
        assert r < MAXOWN, "owner table overflow (the host falls back to step launches)"
        own[w][r] = c
    return own


def prio(c):
    return (c[0] << 16) | (c[1] << 8) | c[2]         # flow_prio: A, then R / Y, then alpha


def wave_program(slots, T):
    """The item sequence of one worker wave (flow_worker): slots in priority order; per level
    the stand-alone finalizes (tiles without updates), then the updates (an A or R tile's last
    update carries its finalize)."""
    slots = sorted([c for c in slots if c is not None], key=prio)
    last = max([max(tile(c, T)[1], tile(c, T)[2]) for c in slots] or [-1])
    prog = []
    for l in range(last + 1):
        for c in slots:
            lo, hi, fin, _ = tile(c, T)
            if fin == l and hi < lo:
                prog.append(("fin", c, l))
        for c in slots:
            lo, hi, fin, _ = tile(c, T)
            if lo <= l <= hi:
                prog.append(("upd", c, l))
    return prog


def needs_and_makes(item, T):
    """Published inputs an item waits for / outputs it publishes (FlowPub slots)."""
    kind, (ty, i, j), l = item
    lo, hi, fin, pub = tile((ty, i, j), T)
    need, make = [], []
    if kind == "fin":                                 # stand-alone finalize
        need.append(("D", fin))
        make.append(("L", i, j) if ty == FT_A else ("X", i, j))   # X(0,c) = D_0 Y(0,c)
        return need, make
    if ty == FT_A:
        need += [("L", i, l), ("L", j, l)]
        if fin == l + 1:                              # merged finalize
            need.append(("D", fin))
            make.append(("L", i, j))
        elif pub and l == hi:
            make.append(("H", i, j))
    elif ty == FT_R:
        need += [("L", i, l), ("X", l, j)]
        if l == hi:                                   # merged finalize X(i,c) = D_i R'''
            need.append(("D", fin))
            make.append(("X", i, j))
    else:
        need += [("X", l, i), ("X", l, T + j)]
    return need, make


def diag_needs(k, T):
    """Diag workgroup, chain step k (waves 5-7 prefetch + chain): what D_k, L(k,k-1), L(k,k-2),
    X(k,k) wait for.  Row 3's band tiles are FT_G tiles, published by their owners in the Gram
    phase at the start of the launch (rows 1-2: the diag workgroup's own)."""
    need = [("G", 3, j) for j in (1, 2, 3)] if k == 3 else []
    if k >= 4:
        need += [("H", k, k - 2), ("H", k, k - 1), ("H", k, k)]
    if k >= 3:
        need.append(("L", k, k - 3))
    return need


def simulate(T, Tp, W, reverse=False):
    own = owner_table(T, Tp, W)
    if reverse:
        own = own[::-1]
    progs = [wave_program(s, T) for s in own]
    done = set()
    # D_0 (the diag's waves 0/1 form tile (0,0), wave 0 factors it) and X(0,0); the Gram phase's
    # FT_G publications (before any wave's items: no inputs)
    done |= {("D", 0), ("X", 0, 0)}
    done |= {("G", c[1], c[2]) for s in own for c in s if c is not None and c[0] == FT_G}
    pos = [0] * len(progs)
    dk = 1
    progress = True
    while progress:
        progress = False
        # diag chain: step k needs the chain's own L(k-1,k-2) etc. (internal) and the band inputs
        while dk < T and all(n in done for n in diag_needs(dk, T)):
            done |= {("D", dk), ("X", dk, dk), ("L", dk, dk - 1)}
            if dk >= 2:
                done.add(("L", dk, dk - 2))
            dk += 1
            progress = True
        for w, prog in enumerate(progs):
            while pos[w] < len(prog):
                need, make = needs_and_makes(prog[pos[w]], T)
                if not all(n in done for n in need):
                    break
                done |= set(make)
                pos[w] += 1
                progress = True
    stuck = [(w, progs[w][pos[w]]) for w in range(len(progs)) if pos[w] < len(progs[w])]
    return dk, stuck, done


@pytest.mark.parametrize("T,Tp", [(1, 1), (2, 2), (3, 1), (4, 2), (5, 3), (9, 1), (37, 2), (47, 2)])
def test_every_tile_owned_once(T, Tp):
    W = 8 * 255
    if ntiles(T, Tp) > W * MAXOWN:
        pytest.skip("host uses the step schedule")
    own = owner_table(T, Tp, W)
    flat = [c for s in own for c in s if c is not None]
    assert len(flat) == len(set(flat)) == ntiles(T, Tp)
    # every output tile of the factorization is produced by someone: L(i,j) i > j, X(i,c)
    made = set()
    for s in own:
        for it in wave_program(s, T):
            made |= set(needs_and_makes(it, T)[1])
    for i in range(T):
        for j in range(i):
            assert ("L", i, j) in made or j >= i - 2, (i, j)   # band finalizes are diag's
        for c in list(range(i)) + [T + y for y in range(Tp)]:
            assert ("X", i, c) in made, (i, c)


@pytest.mark.parametrize("T,Tp,W", [(1, 2, 8), (2, 1, 8), (3, 2, 5), (4, 2, 16), (6, 1, 9), (12, 2, 40),
                                    (37, 2, 2040), (37, 2, 400), (20, 3, 120), (12, 2, 240), (30, 2, 1400)])
@pytest.mark.parametrize("reverse", [False, True])
def test_schedule_runs_to_completion(T, Tp, W, reverse):
    if ntiles(T, Tp) > W * MAXOWN:
        pytest.skip("owner table too small: the host uses the step schedule")
    dk, stuck, done = simulate(T, Tp, W, reverse)
    assert dk == T and not stuck, (dk, stuck[:3])
    # alpha and Z of every row are complete
    for i in range(T):
        for y in range(Tp):
            assert ("X", i, T + y) in done
