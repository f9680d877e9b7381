"""Test-infrastructure oracles (CPU restatements of the reference's hot path).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  See nlp_ref.py (NumPy) and ipm_ref.cpp (C++ IPM, ctypes via ipm_ref.py).
"""
