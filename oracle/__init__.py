"""CPU oracle package -- TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker. Never imported by storb_amd.
"""
