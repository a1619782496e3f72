"""Diagnostic: which graph-lifetime order crashes hipGraphLaunch.

Round 5's knob sweep segfaulted in the first replay of its fifth configuration when each
configuration's session (and its captured fp32 lookahead graphs) was dropped only after the next
session had been created.  Each scenario below runs in a child process with faulthandler on; the
driver prints the child's exit status and the tail of its stderr (the Python stack of a crash).

  python tools/graph_lifetime_probe.py            # every scenario, one child each
  python tools/graph_lifetime_probe.py NAME       # one scenario in this process
"""
import faulthandler
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SCENARIOS = ["small_close_before", "small_buffers_after", "small_graphs_after", "f32_small_sweep"]


def _log(msg):
    print(msg, flush=True)


def _model(n_lf, n_hf, p):
    import numpy as np
    import multi_fidelity_gpflow_amd as M
    from multi_fidelity_gpflow_amd.data import synthetic_multifidelity
    X, Y, _, _ = synthetic_multifidelity(n_lf=n_lf, n_hf=n_hf, p=p)
    d = X.shape[1] - 1
    return M.MultiFidelityGPModel(X, Y, M.SquaredExponential(lengthscales=np.ones(d)),
                                  M.SquaredExponential(lengthscales=np.ones(d)), dtype="float32")


def torch_forkjoin():
    """No library: graphs with a side-stream fork / join (torch matmuls), each dropped only after the
    next one was created and warmed up, as the sweep did."""
    import torch
    a = torch.randn(2048, 2048, device="cuda")
    side = torch.cuda.Stream(priority=-1)
    _ = a @ a   # hipBLASLt's workspace exists before any capture
    with torch.cuda.stream(side):
        _ = a @ a
    torch.cuda.synchronize()
    g_old = None
    for i in range(8):
        g = torch.cuda.CUDAGraph()
        b = torch.empty_like(a)
        with torch.cuda.graph(g):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                c = a @ a
            b.copy_(a @ a.T)
            cur.wait_stream(side)
            b.add_(c)
        g_old = None   # the previous graph dies after the new capture
        g.replay()
        torch.cuda.synchronize()
        g_old = g
        _log(f"torch_forkjoin {i}: ok")


def _sweep(configs, lookahead=True, n=(16384, 2048, 512), order="reassign"):
    """order: "reassign" (round 5: the previous session dies when the next one is assigned, after
    its creation and warm-up, before its capture), "keep" (no session is ever dropped), "after"
    (the previous session is dropped after the next one captured, before its first replay)."""
    import torch
    from multi_fidelity_gpflow_amd.engine import Engine
    torch.cuda.set_device(0)
    eng = Engine.get()
    eng.set_f32_lookahead(lookahead)
    m = _model(*n)
    sess, kept = None, []
    for i, (panel, rv) in enumerate(configs):
        eng.set_f32_panel(panel)
        eng.set_f32_reserve(rv)
        prev = sess
        sess = m.adam_session(0.1, 8, graph=True, graph_chunk=2)
        if order == "reassign":
            prev = None
        elif order == "keep":
            kept.append(prev)
            prev = None
        sess.run(2)
        sess.prepare(4)
        if order == "after":
            prev = None
        sess.sync()
        t0 = time.time()
        sess.run(4)
        sess.sync()
        _log(f"config {i} panel={panel} reserve={rv} stream {sess.stream.cuda_stream:#x}: "
             f"{(time.time() - t0) / 4 * 1e3:.1f} ms/step")


def _small_sweep(variant, count=8):
    """Bisection of the reassign order at a small fp32 size (lookahead on):
      close_before   the previous session's graphs closed before the next session is created
                     (round 5's fix), its buffers dropped after
      graphs_after   the next session created and warmed up, then the previous session's graphs
                     closed (its buffers kept alive), then the capture
      buffers_after  the previous session's graphs closed before the next session is created, its
                     buffers dropped after the next session's warm-up (before the capture)"""
    import torch
    from multi_fidelity_gpflow_amd.engine import Engine
    torch.cuda.set_device(0)
    eng = Engine.get()
    eng.set_f32_lookahead(True)
    m = _model(3584, 512, 64)
    prev, kept = None, []
    for i in range(count):
        if prev is not None and variant in ("close_before", "buffers_after"):
            prev.close()
        sess = m.adam_session(0.1, 8, graph=True, graph_chunk=2)
        sess.run(2)
        if prev is not None:
            if variant == "graphs_after":
                prev.close()
                kept.append(prev)
            prev = None          # close_before / buffers_after: the buffers go here
        sess.prepare(4)
        sess.sync()
        sess.run(4)
        sess.sync()
        _log(f"{variant} {i}: ok")
        prev = sess
        del sess


def small_close_before():
    _small_sweep("close_before")


def small_graphs_after():
    _small_sweep("graphs_after")


def small_buffers_after():
    _small_sweep("buffers_after")


def f32_keep_all():
    _sweep([(6, 32)] * 7, order="keep")


def f32_destroy_after_capture():
    _sweep([(6, 32)] * 7, order="after")


def f32_small_sweep():
    _sweep([(6, 32)] * 8, n=(3584, 512, 64))


def f32_sweep_old():
    _sweep([(4, 32), (6, 32), (8, 32), (4, 48), (8, 48), (2, 32)])


def f32_sweep_same():
    _sweep([(6, 32)] * 6)


def f32_sweep_nolook():
    _sweep([(4, 32), (6, 32), (8, 32), (4, 48), (8, 48), (2, 32)], lookahead=False)


def f32_small_abrb():
    """VERDICT's order at a small fp32 size with the lookahead: capture A, capture B, release A,
    replay B (several rounds)."""
    import torch
    torch.cuda.set_device(0)
    m = _model(3584, 512, 64)
    for i in range(6):
        a = m.adam_session(0.1, 8, graph=True, graph_chunk=2)
        a.run(2)
        a.prepare(4)
        a.run(4)
        b = m.adam_session(0.1, 8, graph=True, graph_chunk=2)
        b.run(2)
        b.prepare(4)
        a.close()
        del a
        b.run(4)
        b.sync()
        _log(f"f32_small_abrb {i}: ok")
        del b


def hip_only():
    """The same orders with the HIP runtime alone (tools/ubench_graph_lifetime.hip), one child per
    mode; stops at the first crash."""
    exe = os.path.join(ROOT, "tools", "ubench_graph_lifetime")
    for mode in (sys.argv[2:] or ["after", "nofork", "samestream", "reassign", "reassign_free", "after_cs",
                                  "reassign_cs"]):
        r = subprocess.run([exe, mode], capture_output=True, text=True, timeout=120)
        _log(f"== hip {mode}: exit {r.returncode}")
        for ln in (r.stdout + r.stderr).splitlines()[-6:]:
            _log("   " + ln)
        if r.returncode not in (0, 1):
            _log("stopping: the child crashed, aborted or timed out")
            sys.exit(3)


def driver():
    outdir = os.path.join(ROOT, "gpurun_out", "graph_probe")
    os.makedirs(outdir, exist_ok=True)
    for name in (sys.argv[2:] or SCENARIOS):
        t0 = time.time()
        with open(os.path.join(outdir, name + ".log"), "w") as f:
            r = subprocess.run([sys.executable, "-u", "-X", "faulthandler", os.path.abspath(__file__), name],
                               stdout=f, stderr=subprocess.STDOUT, timeout=300)
        tail = open(os.path.join(outdir, name + ".log")).read().splitlines()[-25:]
        _log(f"== {name}: exit {r.returncode} after {time.time() - t0:.1f} s")
        for ln in tail:
            _log("   " + ln)
        if r.returncode not in (0, 1):
            # a crash, abort or time limit: nothing more runs on the GPU in this call
            _log("stopping: the child crashed, aborted or timed out")
            sys.exit(3)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "--hip":
        hip_only()
    elif len(sys.argv) > 1 and sys.argv[1] != "--all":
        faulthandler.enable()
        globals()[sys.argv[1]]()
    else:
        driver()
