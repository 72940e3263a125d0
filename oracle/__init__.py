"""oracle/ -- CPU checkers for the CRC-32 path.  TEST INFRASTRUCTURE ONLY.

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg.  The product package rpc_amd never imports anything from here.
"""
