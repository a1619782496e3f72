"""Where the Goku train (1000 Adam steps) + predict_f wall-clock goes beyond the steps themselves:
session set-up, graph capture, replay, finish, predict (GPU box, repo root)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import load_goku, make_model  # noqa: E402


def clock():
    torch.cuda.synchronize()
    return time.perf_counter()


torch.cuda.set_device(0)
X, Y, Xt, _ = load_goku()
for rep in range(3):
    m = make_model(X, Y)
    m._device_data()
    t0 = clock()
    sess = m.adam_session(0.1, 1000, True, 50)
    t1 = clock()
    sess.prepare(1000)
    t2 = clock()
    sess.run(1000)
    t3 = clock()
    sess.finish()
    t4 = clock()
    mean, var = m.predict_f(Xt)
    t5 = clock()
    print(f"rep {rep}: session {1e3 * (t1 - t0):.1f} ms, capture {1e3 * (t2 - t1):.1f} ms, 1000 steps "
          f"{1e3 * (t3 - t2):.1f} ms, finish {1e3 * (t4 - t3):.1f} ms, predict {1e3 * (t5 - t4):.1f} ms; "
          f"total {1e3 * (t5 - t0):.1f} ms")
