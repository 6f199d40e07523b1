"""ORACLE — test infrastructure only.  CPU fp32 restatement of the reference
training step, pinned against golden vectors from the reference itself
(tests/golden/).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import it; the HIP product path never does."""
