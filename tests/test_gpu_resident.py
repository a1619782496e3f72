"""Resident workspace mode (include/mfgp.h mfgp_set_resident): a value+grad call whose
workspace the previous fp64 LML call on the handle left set up for the same problem skips the flow's
set-up launch.  Every interleaving below must give exactly the result of a non-resident call:
repeated resident calls, a value-only call in between (it leaves no set-up behind), a switch to
another problem on the same workspace and back, and a timed-out flow (the abort path) followed by a
resident call."""
import numpy as np
import pytest
import torch

from multi_fidelity_gpflow_amd._lib import MFGP_FLOW_TIMEOUT
from multi_fidelity_gpflow_amd.engine import Engine

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = Engine.get()
    e.set_flow(True)
    yield e
    e.set_flow_timeout_us(50000)


def _theta(d, seed):
    rng = np.random.default_rng(seed)
    return np.concatenate([[0.5 + rng.random()], 0.5 + rng.random(d), [0.1 + rng.random()], 0.5 + rng.random(d),
                           [0.5 + rng.random()], [1e-3]])


def test_resident_matches_nonresident_under_interleavings(goku, eng):
    if not eng.flow_runs(goku["X"].shape[0]):
        pytest.skip("persistent Cholesky not available on this device")
    dev = eng.device
    X = torch.tensor(goku["X"], dtype=torch.float64, device=dev)
    Ya = torch.tensor(goku["Y"], dtype=torch.float64, device=dev)
    Yb = torch.tensor(goku["Y"][:, :40], dtype=torch.float64, device=dev).contiguous()
    d = X.shape[1] - 1
    th = torch.tensor(_theta(d, 5), dtype=torch.float64, device=dev)
    n = X.shape[0]
    ws = eng.private_workspace(max(eng.gpr_workspace_bytes(n, 64, d), eng.gpr_workspace_bytes(n, 40, d)))

    def call(Y, grad=True, w=ws):
        out, info = eng.gpr_lml(X, Y, th, want_grad=grad, ws=w)
        torch.cuda.synchronize()
        return out.cpu().numpy().copy(), int(info.item())

    # references: non-resident calls on a workspace of their own
    ref_a, ia = call(Ya, w=eng.private_workspace(ws.numel()))
    ref_b, ib = call(Yb, w=eng.private_workspace(ws.numel()))
    ref_v, iv = call(Ya, grad=False, w=eng.private_workspace(ws.numel()))
    assert ia == ib == iv == 0
    with eng.resident():
        seq = [("a", call(Ya)), ("a", call(Ya)), ("a", call(Ya)),   # the 2nd and 3rd skip the set-up
               ("v", call(Ya, grad=False)), ("a", call(Ya)),         # value-only in between
               ("b", call(Yb)), ("b", call(Yb)), ("a", call(Ya)), ("a", call(Ya))]   # problem switch
        eng.set_flow_timeout_us(0)
        try:
            _, info_t = call(Ya)                                     # aborted flow
        finally:
            eng.set_flow_timeout_us(50000)
        assert info_t == MFGP_FLOW_TIMEOUT
        seq += [("a", call(Ya)), ("a", call(Ya))]
    refs = {"a": ref_a, "b": ref_b, "v": ref_v}
    for i, (k, (o, info)) in enumerate(seq):
        assert info == 0, (i, k, info)
        nv = 1 if k == "v" else o.size   # a value-only call writes out[0] only
        np.testing.assert_array_equal(o[:nv], refs[k][:nv], err_msg=f"call {i} ({k})")
