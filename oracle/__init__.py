"""Oracle package: CPU restatement of the hot path. TEST INFRASTRUCTURE ONLY.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  The product package never imports it.
"""
