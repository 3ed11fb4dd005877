"""Drop-in replacement for the reference's Cython module ``fisher_cython_parallel``
(statistics/fisher/fisher_cython_parallel.pyx), imported by FisherExactScoreStat.py:19
as ``from quick.statistic.fisher_cython_parallel import fisher_exact_tester``.
Place this directory where that import resolves."""
from gdscan.fet import fisher_exact_tester  # noqa: F401
