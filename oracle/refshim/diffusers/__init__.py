"""Minimal stand-in for the parts of diffusers 0.32.2 that the reference's
latentsync/models/* import.  TEST INFRASTRUCTURE ONLY: used by
oracle/make_golden.py to import the read-only reference in this container and
emit golden vectors.  Never imported by the product path."""
