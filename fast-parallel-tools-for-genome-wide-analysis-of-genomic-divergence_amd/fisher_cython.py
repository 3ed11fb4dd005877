"""Drop-in replacement for the reference's serial Cython module ``fisher_cython``
(statistics/fisher/fisher_cython.pyx; FisherExactScoreStat.py:18)."""
from gdscan.fet import fisher_exact_tester_serial as fisher_exact_tester  # noqa: F401
