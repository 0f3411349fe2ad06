"""Multi-GPU paths: corpus-sharded top-K, table-sharded gather, DP averaging."""
from .sharded import (ShardedFlatIPIndex, all_gather_candidates, allreduce_mean_, owner_of, shard_range,
                      sharded_gather_rows, sharded_inbatch_step, sharded_topk)

__all__ = ["ShardedFlatIPIndex", "all_gather_candidates", "allreduce_mean_", "owner_of", "shard_range",
           "sharded_gather_rows", "sharded_inbatch_step", "sharded_topk"]
