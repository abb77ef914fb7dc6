"""Process bootstrap: one process per GPU, host control plane + RCCL data plane."""
from .dist import DistEnv, env, init, init_ctrl, select_device  # noqa: F401
