"""oracle -- TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference's render path used as the parity checker
(tests/, __graft_entry__.smoke) and as bench.py's cpu_baseline.  Never imported by
the product package scenedino_amd.
"""
