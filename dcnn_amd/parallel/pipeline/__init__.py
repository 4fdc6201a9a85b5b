"""Pipeline parallelism: partitioners, stage event loop, coordinators (sync / semi-async),
native control plane (TCP / in-process) and the RCCL point-to-point data plane."""
from .config import Endpoint, StageConfig  # noqa: F401
from .coordinator import Coordinator, DistributedCoordinator, InProcessCoordinator, PipelineError  # noqa: F401
from .messages import CommandType  # noqa: F401
from .partitioner import (CostPartitioner, FlopPartitioner, NaivePartitioner, Partitioner,  # noqa: F401
                          balanced_split, create_partitioner)
from .stage import PipelineStage, flat_state, load_flat_state  # noqa: F401
from .train import train_model, train_semi_async_epoch, validate_semi_async_epoch  # noqa: F401
from .transport import LocalTransport, MessageTransport, P2PTransport, make_groups  # noqa: F401
from .worker import NetworkStageWorker  # noqa: F401
