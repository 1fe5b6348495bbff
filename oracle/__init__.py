"""Python wrapper of the CPU oracle (oracle/cvr_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.
"""
from .oracle import *  # noqa: F401,F403
