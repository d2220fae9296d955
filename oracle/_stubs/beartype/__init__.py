"""Stand-in for ``beartype`` (runtime type checking only; absent here).  TEST INFRASTRUCTURE:
lets tests/golden/make_golden_bsr.py import the reference BS-Roformer module."""


def beartype(fn):
    return fn
