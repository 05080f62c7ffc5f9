"""ORACLE (test infrastructure only): CPU restatement of the reference crosscoder step.
Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg."""
