"""CPU oracle for the RRDB-23 + CEM ×4 hot path — TEST INFRASTRUCTURE ONLY.

This package is a from-scratch CPU restatement of the reference's algorithm (PyTorch-CPU ops for the fp32 convolution
graph, NumPy float64 for the CEM filter design).  It is imported only by `tests/`, `__graft_entry__.smoke()` and
`bench.py`'s `cpu_baseline` leg, and there only as the CHECKER.  The product path
(`explorable-super-resolution_old_amd/esr_amd`) never imports it and fails loudly when its HIP library is missing.

Pinning: every function here is checked against golden vectors produced by importing the reference itself in the build
container (`tests/golden/make_golden.py`, committed together with its .npz outputs; see tests/test_oracle_golden.py).
"""
