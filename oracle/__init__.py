"""TEST INFRASTRUCTURE ONLY: the CPU parity oracle (see oracle/oracle.py)."""
