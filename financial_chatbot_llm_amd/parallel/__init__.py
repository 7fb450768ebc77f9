"""Distributed execution: process groups (RCCL over xGMI), TP sharding, collectives."""
from .dist import ParallelState, init_distributed, state

__all__ = ["ParallelState", "init_distributed", "state"]
