"""CPU oracle for the multi-fidelity GP hot path — TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this package, and only as the checker / the timed CPU baseline.
The product path (``multi_fidelity_gpflow_amd``) never imports it.
"""
