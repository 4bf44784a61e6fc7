"""CPU oracle for dpwa's pairwise-averaging hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import anything under ``oracle/``, and only as the checker (or the timed CPU
baseline).  The product package ``dpwa_amd`` never imports it and has no CPU
fallback: without its HIP library it raises.

Contents (each function cites the reference file:line it restates):
  lerp.py     fp32 / bf16 averaging (dpwa/adapters/pytorch.py:68), numpy + the C build
              of dpwa_oracle.c (oracle/_build/libdpwa_oracle.so, built by oracle/Makefile)
  policy.py   interpolation factor, divergence scaling, clock (dpwa/dpwa.py:101-156,
              dpwa/interpolation.py:8-33) and TxThread peer choice + flow control
              (dpwa/conn.py:178-317) driven by CPython's own MT19937 (random.Random)
  gossip.py   a lock-step G-learner gossip simulation composed from the two above

Pinning: tests/test_oracle.py checks every function here against the golden
fixtures in tests/golden/, which tests/golden/make_golden.py produced by running
the reference itself in the build container.  The bf16 lerp is pinned to
torch-eager bf16 arithmetic (the reference has no bf16 path, pytorch.py:11-14).
"""
