"""MI355X-native distributed hyperparameter-search engine.

A re-design (not a port) of sanjita2911/CS230-distributed-machine-learning: the
``MLTaskManager`` client API and job-result JSON are kept, while the
Flask/Kafka/Redis master-scheduler-worker stack collapses onto one node where each
MI355X GPU is a worker rank (``torch.distributed`` over RCCL/xGMI) and the fit hot
paths are hand-written HIP kernels for gfx950 (see SURVEY.md and README.md).
"""
__version__ = "0.3.0"

from .client.core import MLTaskManager  # noqa: E402

__all__ = ["MLTaskManager", "__version__"]
