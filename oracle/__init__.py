"""TEST INFRASTRUCTURE ONLY.

CPU restatements of the reference algorithms (oracle/bp_oracle.c for
ldpc_jossy/src/c_ldpc.c, oracle/sparc_ref.py for sparc_public/sparc.py and
sparc_sophie/sparc_new.py) used as the parity checker by tests/, by
__graft_entry__.smoke(), and as the timed CPU baseline in bench.py.  The
product (ldpc_sparc_amd/) never imports anything from here.
"""
