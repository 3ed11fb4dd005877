"""Drop-in replacement for the reference's Cython module ``css_cython_parallel``
(statistics/css/css_cython_parallel.pyx), imported by CategoryClusterSeparationStat.py:19."""
from gdscan.css import cluster_separation_scorer  # noqa: F401
