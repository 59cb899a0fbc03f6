from .core import MLTaskManager

__all__ = ["MLTaskManager"]
