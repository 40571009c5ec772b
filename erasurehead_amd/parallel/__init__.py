"""Distribution (L7): process topology, worker placement, RCCL/gloo p2p, native arrival collector."""
from .collector import ArrivalCollector
from .dist import DistEnv, init_distributed
from .placement import place_workers, workers_by_rank
