"""ORACLE package — test infrastructure only (see nslam_oracle.py header)."""
