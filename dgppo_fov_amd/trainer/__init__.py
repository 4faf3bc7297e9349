from .data import Rollout  # noqa: F401
