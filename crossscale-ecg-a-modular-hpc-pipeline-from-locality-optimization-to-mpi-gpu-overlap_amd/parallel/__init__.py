"""Distributed layer: launcher env shim, RCCL/gloo process group, FedAvg on flat buffers, overlap, DDP."""
from .env import init_distributed, get_context, shutdown_distributed, setup_device, barrier, DistContext  # noqa: F401
from .fedavg import (Communicator, broadcast_model, fedavg_allreduce, mpi_avg, allreduce_mean_,  # noqa: F401
                     weighted_fedavg_, DelayedFedAvg)
from .seqpar import (shard_bounds, halo_exchange, SeqShardedConv1d, seq_global_avg_pool,  # noqa: F401
                     SeqParallelTinyECG, allreduce_seq_grads_)
