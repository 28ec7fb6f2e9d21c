"""Decomposition math and the torch.distributed -> RCCL bootstrap."""
from .bootstrap import dist_info, nccl_unique_id  # noqa: F401
from .decomposition import SlabDecomposition, balanced_split  # noqa: F401
