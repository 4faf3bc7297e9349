"""CPU oracle: NumPy restatement of the reference DGPPO hot paths.

TEST INFRASTRUCTURE ONLY.  Nothing in `dgppo_fov_amd/` imports this package; only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it, and only as the checker /
the timed CPU baseline — never as a fallback for the product path.

Parity status: **parity unpinned** against the reference itself.  The reference (Tw6249/dgppo_fov,
pure JAX) ships no tests, golden vectors or fixtures, and JAX/flax/jraph/tfp
are not installed in this image, so the reference cannot be executed to generate any.  Each
function below restates the reference source line by line (file:line cited in its docstring) and
is pinned only by hand-derived known-answer tests (tests/test_oracle_kat.py) and by the committed
fixtures in tests/golden/ (produced by this restatement; see tests/golden/make_golden.py).
"""
