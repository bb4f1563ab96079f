"""CPU oracle for the hash-join probe / compaction hot path. TEST INFRASTRUCTURE ONLY:
imported by tests/, __graft_entry__.smoke() and bench.py cpu_baseline, never by the product."""
