"""Test-only CPU oracle for the FI-ODE hot path (see fiode_oracle.py header)."""
