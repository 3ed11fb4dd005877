"""gdscan -- MI355X-native genomic-divergence window scanner (FET + CSS).

Host-side mirror of the reference's hot path:
  fet.fisher_exact_tester        <- statistics/fisher/fisher_cython_parallel.pyx:14-15
  css.cluster_separation_scorer  <- statistics/css/css_cython_parallel.pyx:14-15
  stats.FisherExactScoreStatUnsplittable / CategoryClusterSeparationStatUnsplittable
                                 <- statistics/*.py _compute
  shard.plan_shards / gather_tracks  multi-GPU chromosome sharding
All compute runs in lib/libgdscan.so (HIP, gfx950); importing this package fails
loudly when that library is missing.
"""
from ._lib import GdError, lib, check  # noqa: F401
from . import fet, css, shard, stats  # noqa: F401

__all__ = ["GdError", "fet", "css", "shard", "stats", "lib", "check"]
