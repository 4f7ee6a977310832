"""CPU oracle package -- TEST INFRASTRUCTURE ONLY (see u2_oracle.py header)."""
