"""Probe (GPU box, repo root): the cost of a step graph's FIRST replay on the Goku headline step.

The driver times `bench.py --steps 20 --warmup 5`: the timed region is the first replay of a
20-step graph captured just before it (prepare).  This times run(20) per step for
  fresh    a newly captured graph, replayed for the first time (the driver's case);
  upload   the same after hipGraphUpload of the new exec on the session stream (by hand here);
  replay2  a newly captured graph whose first replay ran untimed just before.
Prints one JSON line: ms per step per mode, every repetition.
    python tools/graph_first_replay_probe.py [REPS]"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from multi_fidelity_gpflow_amd import models  # noqa: E402


def main(reps):
    dev = torch.device("cuda:0")
    X, Y, _, _ = bench.broadcast_inputs(0, 1, dev)
    model = bench.make_model(X, Y, None)
    hip = ctypes.CDLL("libamdhip64.so")
    sess = model.adam_session(0.1, 5 + reps * 3 * 40, graph=True, graph_chunk=50)
    sess.run(5)
    sess.sync()

    def timed(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        sess.run(n)
        sess.sync()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    res = {"fresh": [], "upload": [], "replay2": []}
    for _ in range(reps):
        for mode in res:
            models._retire_graphs({20: sess.runner.graphs.pop(20)} if 20 in sess.runner.graphs else {})
            sess.prepare(20)
            if mode == "upload":
                g = sess.runner.graphs[20]
                rc = hip.hipGraphUpload(ctypes.c_void_p(g.raw_cuda_graph_exec()),
                                        ctypes.c_void_p(sess.stream.cuda_stream))
                assert rc == 0, rc
                sess.sync()
            if mode == "replay2":
                timed(20)
            res[mode].append(round(timed(20), 4))
    sess.finish()
    print(json.dumps({"ms_per_step": res, "mean": {k: round(sum(v) / len(v), 4) for k, v in res.items()}}))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 5)
