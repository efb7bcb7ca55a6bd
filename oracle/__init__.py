"""Test-only CPU oracle for the Chemeleon sampling path (see chemeleon_oracle.py).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this package. The product path (chemeleon_amd) never does.
"""
