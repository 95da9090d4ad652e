"""CPU oracle for picotron's decoder-layer hot path -- test infrastructure only (see picotron_oracle.py)."""
