"""Compatibility import surface: ``from distributed_ml import MLTaskManager``.

Same public name as the reference pip package (DistributedLibrary/src/distributed_ml/
__init__.py:1-3); implemented by ``cs230_distributed_machine_learning_amd.client``.
"""
from cs230_distributed_machine_learning_amd.client.core import MLTaskManager

__all__ = ["MLTaskManager"]
