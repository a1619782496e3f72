"""Where the train + predict wall-clock goes beyond the steps themselves: model construction,
session set-up, graph capture, replay, finish, predict (GPU box, repo root).
    python tools/tp_breakdown.py [goku|hbs]   (goku: 1000 Adam steps; hbs: the reference test's 100)"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import HBS, load_goku, make_model  # noqa: E402


def clock():
    torch.cuda.synchronize()
    return time.perf_counter()


torch.cuda.set_device(0)
which = sys.argv[1] if len(sys.argv) > 1 else "goku"
if which == "hbs":
    from multi_fidelity_gpflow_amd.data import PowerSpecs, multifidelity_training_set
    ps = PowerSpecs()
    ps.read_from_txt(HBS)
    X, Y, Xt, _ = multifidelity_training_set(ps)
    steps = 100
else:
    X, Y, Xt, _ = load_goku()
    steps = 1000
for rep in range(4):
    tm = clock()
    m = make_model(X, Y)
    m._device_data()
    t0 = clock()
    sess = m.adam_session(0.1, steps, True, 50)
    t1 = clock()
    sess.prepare(steps)
    t2 = clock()
    sess.run(steps)
    t3 = clock()
    sess.finish()
    t4 = clock()
    mean, var = m.predict_f(Xt)
    t5 = clock()
    print(f"{which} rep {rep}: model {1e3 * (t0 - tm):.2f} ms, session {1e3 * (t1 - t0):.2f} ms, capture "
          f"{1e3 * (t2 - t1):.2f} ms, {steps} steps {1e3 * (t3 - t2):.2f} ms, finish {1e3 * (t4 - t3):.2f} ms, "
          f"predict {1e3 * (t5 - t4):.2f} ms; total {1e3 * (t5 - tm):.2f} ms", flush=True)
