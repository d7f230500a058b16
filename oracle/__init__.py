"""ORACLE — test infrastructure only; never on the product path.

CPU restatement of the reference hot path (Shashank8834/multimodal-fl-security
@ 2025-12-26).  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this package, and only as the
checker / the timed CPU baseline.

Pinning status: the reference is pure Python over torch/numpy and running or
importing it was refused in this environment, so the oracle
re-types each cited function with the SAME torch/numpy calls in the SAME order
on this image's pinned versions (torch 2.10.0+rocm7.0, numpy 2.2.6).  It is
pinned against the reference's own tests (tests/test_defenses.py,
tests/test_attacks.py property tests, restated in tests/test_oracle.py) and
against the op-level semantics those calls have (numpy pairwise summation,
torch's cascade outer sum, IEEE division) — the reference holds no
known-answer vectors for this path.
"""
