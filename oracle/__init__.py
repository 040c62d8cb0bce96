"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (parity checker, never the product path).

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
Parity is pinned by golden vectors captured from the reference itself
(tests/golden/make_golden.py -> tests/golden/*.npz).
"""
