"""Data parallelism: one process per GPU, RCCL all-reduce of flat gradient buckets overlapped
with backward (the only parallelism of the reference: MirroredStrategy towers)."""
from .dist import DistContext, init_distributed, get_context, shutdown
from .bucketer import GradBucketer
from .launcher import spawn, free_port

__all__ = ["DistContext", "init_distributed", "get_context", "shutdown", "GradBucketer", "spawn",
           "free_port"]
