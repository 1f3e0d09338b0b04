"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the `Bls` hot path.

Nothing in the product (`lambda_ethereum_consensus_amd/`, `libmbls.so`) may import,
link or execute anything under `oracle/`.  Only `tests/`, `__graft_entry__.smoke()`
and `bench.py`'s `cpu_baseline` leg use it, and only as the checker.
"""
