"""Drop-in replacement for the reference's serial Cython module ``css_cython``
(statistics/css/css_cython.pyx; CategoryClusterSeparationStat.py:18)."""
from gdscan.css import cluster_separation_scorer_serial as cluster_separation_scorer  # noqa: F401
