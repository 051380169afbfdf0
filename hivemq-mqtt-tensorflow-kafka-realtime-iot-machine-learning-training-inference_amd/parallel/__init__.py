"""Multi-GPU execution: RCCL data parallelism and shard-by-key helpers."""
from .dp import (DistEnv, allreduce_max, allreduce_sum_, barrier, broadcast_, init_from_env,  # noqa: F401
                 shard_by_key, shard_range, shutdown)
