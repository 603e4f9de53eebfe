"""ORACLE — TEST INFRASTRUCTURE ONLY.

A CPU restatement of the reference's contraction path (graph bookkeeping + einsum equation
builders + a plain numpy pairwise tensordot executor + the greedy L·M·R sandwich), written
from reading /root/reference as text; each function cites the reference file:line it follows.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package,
and only as the checker / the timed CPU baseline — never as the product path.

Parity status: the reference Python could not be executed in this pipeline (import/run of
/root/reference was denied); `opt_einsum` (the reference's path/pairwise
library, unpinned, not vendored) is not installed.  The reference's own tests hold no golden
values (tests/test_probabilities.py only prints, or asserts P(a|b)=P(ab)/P(b)).  Therefore this
oracle is "parity unpinned" with respect to reference-produced vectors; it is pinned instead by
  * hand-derived bookkeeping fixtures for small graphs (tests/golden/bookkeeping_cases.json),
  * semantic known-answer tests (unitarity => sum |amp|^2 = 1, identity cores => product state,
    projector sandwich == |amp|^2, split+merge == unsplit, conditional = joint / marginal).
"""
